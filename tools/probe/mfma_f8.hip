// Probe: operand lane map and scale semantics of v_mfma_scale_f32_32x32x64_f8f6f4 with
// e4m3 operands, and the output format of v_cvt_pk_fp8_f32 on gfx950 (diagnostic tool).
// Hypothesis H: lane l holds A[l & 31][32 (l >> 5) + j] and B[32 (l >> 5) + j][l & 31] in
// byte j = 0..31 of its 8-VGPR operand; C/D as the bf16 32x32 form (col = l & 31,
// row = (r & 3) + 8 (r >> 2) + 4 (l >> 5)); lane l's E8M0 scale byte scales its own
// 32-element block.  Random small integers (exact in e4m3), host reference in double.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__host__ __device__ unsigned char e4m3(int v) {  // small integers -2..2 -> OCP e4m3fn bits
    switch (v) {
        case 1: return 0x38;
        case 2: return 0x40;
        case -1: return 0xB8;
        case -2: return 0xC0;
        default: return 0x00;
    }
}

__global__ void k(const signed char *A, const signed char *B, float *out, int sa, int sb,
                  const int *lsa, const int *lsb) {
    int l = threadIdx.x;
    if (lsa) {
        sa = lsa[l];
        sb = lsb[l];
    }
    unsigned char ab[32], bb[32];
    for (int j = 0; j < 32; ++j) {
        ab[j] = e4m3(A[(l & 31) * 64 + 32 * (l >> 5) + j]);
        bb[j] = e4m3(B[(32 * (l >> 5) + j) * 32 + (l & 31)]);
    }
    i32x8 a, b;
    for (int w = 0; w < 8; ++w) {
        a[w] = ab[4 * w] | (ab[4 * w + 1] << 8) | (ab[4 * w + 2] << 16) | (ab[4 * w + 3] << 24);
        b[w] = bb[4 * w] | (bb[4 * w + 1] << 8) | (bb[4 * w + 2] << 16) | (bb[4 * w + 3] << 24);
    }
    f32x16 c;
    for (int r = 0; r < 16; ++r) c[r] = 0.f;
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, sa, 0, sb);
    for (int r = 0; r < 16; ++r) {
        int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31;
        out[row * 32 + col] = c[r];
    }
}

__global__ void kcvt(const float *in, unsigned *out) {
    int l = threadIdx.x;
    out[l] = (unsigned)__builtin_amdgcn_cvt_pk_fp8_f32(in[2 * l], in[2 * l + 1], 0, false);
}

int main() {
    signed char hA[32 * 64], hB[64 * 32];
    srand(7);
    for (int i = 0; i < 32 * 64; ++i) hA[i] = (signed char)(rand() % 5 - 2);
    for (int i = 0; i < 64 * 32; ++i) hB[i] = (signed char)(rand() % 5 - 2);
    signed char *dA, *dB;
    float *dO, hO[1024];
    (void)hipMalloc(&dA, sizeof(hA));
    (void)hipMalloc(&dB, sizeof(hB));
    (void)hipMalloc(&dO, 4096);
    (void)hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    (void)hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
    const int scales[3][2] = {{127, 127}, {128, 127}, {126, 129}};  // E8M0: 2^(s - 127)
    for (int t = 0; t < 3; ++t) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dO, scales[t][0], scales[t][1],
                           (const int *)0, (const int *)0);
        (void)hipMemcpy(hO, dO, 4096, hipMemcpyDeviceToHost);
        const double f = ldexp(1.0, scales[t][0] - 127) * ldexp(1.0, scales[t][1] - 127);
        double err = 0, mag = 0;
        for (int i = 0; i < 32; ++i)
            for (int j = 0; j < 32; ++j) {
                double s = 0;
                for (int kk = 0; kk < 64; ++kk) s += (double)hA[i * 64 + kk] * hB[kk * 32 + j];
                err = fmax(err, fabs(s * f - hO[i * 32 + j]));
                mag = fmax(mag, fabs(s * f));
            }
        printf("scales (%d,%d): max |err| %g (max |ref| %g) %s\n", scales[t][0], scales[t][1], err,
               mag, err == 0 ? "H CONFIRMED" : "MISMATCH");
    }
    int hsa[64], hsb[64];
    for (int l = 0; l < 64; ++l) {
        hsa[l] = 125 + rand() % 5;
        hsb[l] = 125 + rand() % 5;
    }
    int *dsa, *dsb;
    (void)hipMalloc(&dsa, 256);
    (void)hipMalloc(&dsb, 256);
    (void)hipMemcpy(dsa, hsa, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(dsb, hsb, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dO, 0, 0, (const int *)dsa, (const int *)dsb);
    (void)hipMemcpy(hO, dO, 4096, hipMemcpyDeviceToHost);
    double err = 0, mag = 0;
    for (int i = 0; i < 32; ++i)
        for (int j = 0; j < 32; ++j) {
            double s = 0;
            for (int kk = 0; kk < 64; ++kk) {
                const int la = i + 32 * (kk >> 5), lb = j + 32 * (kk >> 5);
                s += (double)hA[i * 64 + kk] * ldexp(1.0, hsa[la] - 127) * hB[kk * 32 + j] *
                     ldexp(1.0, hsb[lb] - 127);
            }
            err = fmax(err, fabs(s - hO[i * 32 + j]));
            mag = fmax(mag, fabs(s));
        }
    printf("per-lane block scales: max |err| %g (max |ref| %g) %s\n", err, mag,
           err < 1e-6 * mag ? "CONFIRMED" : "MISMATCH");
    FILE *fo = fopen("gpurun_out/mfma_f8_dump.bin", "wb");
    if (fo) {
        fwrite(hA, 1, sizeof(hA), fo);
        fwrite(hB, 1, sizeof(hB), fo);
        fwrite(hsa, 4, 64, fo);
        fwrite(hsb, 4, 64, fo);
        fwrite(hO, 4, 1024, fo);
        fclose(fo);
    }
    float hin[128];
    unsigned hout[64];
    const float vals[8] = {1.f, -1.f, 2.f, 0.5f, 448.f, 0.0625f, 3.5f, 1e-3f};
    for (int i = 0; i < 128; ++i) hin[i] = vals[i % 8];
    float *din;
    unsigned *dout;
    (void)hipMalloc(&din, 512);
    (void)hipMalloc(&dout, 256);
    (void)hipMemcpy(din, hin, 512, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kcvt, dim3(1), dim3(64), 0, 0, din, dout);
    (void)hipMemcpy(hout, dout, 256, hipMemcpyDeviceToHost);
    printf("cvt_pk_fp8_f32 (1,-1)->%08x (2,0.5)->%08x (448,1/16)->%08x (3.5,1e-3)->%08x\n", hout[0],
           hout[1], hout[2], hout[3]);
    return 0;
}
