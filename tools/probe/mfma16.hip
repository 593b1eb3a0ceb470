// Probe: operand lane map of v_mfma_f32_16x16x16_bf16 (diagnostic tool).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__device__ short bf(float f) { return (short)(__float_as_uint(f) >> 16); }
__global__ void k(float *out, int mode) {
  int l = threadIdx.x;
  s16x4 a, b;
  for (int e = 0; e < 4; ++e) {
    // A element (lane l, e) = 1 + l*4+e (tag) when mode 0; B = "one-hot" on k = lane-elem position
    a[e] = bf(mode == 0 ? (float)(l * 4 + e + 1) : ((l & 15) == 3 ? 1.f : 0.f));
    b[e] = bf(mode == 0 ? (((l & 15) == 0 && e == 0 && (l >> 4) == 0) ? 1.f : 0.f) : (float)(l * 4 + e));
  }
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = c[r];
}
int main() {
  float *d; hipMalloc(&d, 256 * 4); float h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    printf("mode %d:", mode);
    for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) if (h[l * 4 + r] != 0) printf(" (l%d r%d)=%g", l, r, h[l * 4 + r]);
    printf("\n");
  }
  return 0;
}
