// Probe: sd_code_frags values on device vs exact math (diagnostic tool).
#include "../../scenedino_amd/csrc/sdhip_render.h"
#include <stdio.h>
#include <math.h>
extern "C" void sd_set_error(const char *) {}
__global__ void k(float *out, float x, float y, float z) {
  const int l = threadIdx.x, g = l >> 4;
  const float v[3] = {x, y, z};
  bf16x8 f0; sd_s16x4 f1;
  sd_code_frags<bf16x8, sd_s16x4, __bf16>(v, g, f0, f1);
  for (int e = 0; e < 8; ++e) out[l * 12 + e] = (float)f0[e];
  for (int e = 0; e < 4; ++e) out[l * 12 + 8 + e] = __uint_as_float(((uint32_t)(uint16_t)f1[e]) << 16);
}
int main() {
  float *d; (void)hipMalloc(&d, 64 * 12 * 4); float h[64 * 12];
  float v[3] = {0.3f, -0.7f, 0.45f};
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, v[0], v[1], v[2]);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int g = 0; g < 4; ++g) {
    printf("g%d:", g);
    for (int e = 0; e < 12; ++e) printf(" %.4f", h[(16 * g) * 12 + e]);
    printf("\n   ref:");
    if (g < 3) for (int e = 0; e < 12; ++e) { int f = e < 8 ? e / 2 : 4 + (e - 8) / 2, ph = e & 1; printf(" %.4f", sin(v[g] * 1.5 * pow(2, f) + ph * M_PI / 2)); }
    printf("\n");
  }
  return 0;
}
