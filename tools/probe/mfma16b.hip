// Probe: v_mfma_f32_16x16x16_bf16 k-order of A vs B (diagnostic tool).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void k(const float *A, const float *B, float *out) {
  int l = threadIdx.x;
  s16x4 a, b;
  for (int e = 0; e < 4; ++e) {
    a[e] = (short)(__float_as_uint(A[l * 4 + e]) >> 16);
    b[e] = (short)(__float_as_uint(B[l * 4 + e]) >> 16);
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
  float hA[256], hB[256], hO[256];
  for (int i = 0; i < 256; ++i) { hA[i] = (float)((i * 37) % 17) - 8; hB[i] = (float)((i * 53) % 13) - 6; }
  float *dA, *dB, *dO; (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dO, 1024);
  (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dO);
  (void)hipMemcpy(hO, dO, 1024, hipMemcpyDeviceToHost);
  // hypothesis H1: A[i][4g+e] = a(lane i+16g, e), B[4g+e][j] = b(lane j+16g, e)
  double err1 = 0, err2 = 0;
  for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
    int row = 4 * (l >> 4) + r, col = l & 15;
    double s1 = 0, s2 = 0;
    for (int g = 0; g < 4; ++g) for (int e = 0; e < 4; ++e) {
      s1 += hA[(row + 16 * g) * 4 + e] * hB[(col + 16 * g) * 4 + e];
      // H2: A k = 4g+e, B k = g + 4e
      int kk = 4 * g + e, gb = kk % 4, eb = kk / 4;
      s2 += hA[(row + 16 * g) * 4 + e] * hB[(col + 16 * gb) * 4 + eb];
    }
    err1 += fabs(s1 - hO[l * 4 + r]); err2 += fabs(s2 - hO[l * 4 + r]);
  }
  printf("H1 err %g  H2 err %g  sample out %g\n", err1, err2, hO[5]);
  return 0;
}
