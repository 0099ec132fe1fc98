// Verifies the lane map assumed for v_mfma_scale_f32_32x32x64_f8f6f4 with FP4 (e2m1) A and B
// and unit E8M0 scales (127):
//   A: lane l, nibble j (j even = low nibble of byte j/2) -> A[l&31][32*(l>>5)+j]
//   B: lane l, nibble j                                   -> B[32*(l>>5)+j][l&31]
//   C: lane l, reg r -> C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]   (shape-determined)
// Data: random e2m1 codes (all 16), asymmetric, so a swapped nibble order, half or row/col
// shows up as mismatches.  Prints the count for the low-nibble-first and high-first packings.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__global__ void k(const unsigned char* A, const unsigned char* B, float* C, int hi_first) {
  const int l = threadIdx.x, h = l >> 5, r = l & 31;
  v8i a = {0}, b = {0};
  unsigned char* pa = (unsigned char*)&a;
  unsigned char* pb = (unsigned char*)&b;
  for (int j = 0; j < 32; ++j) {
    const unsigned ca = A[r * 64 + 32 * h + j], cb = B[(32 * h + j) * 32 + r];
    const int sh = ((j & 1) ^ hi_first) * 4;
    pa[j >> 1] |= ca << sh;
    pb[j >> 1] |= cb << sh;
  }
  v16f c = {0};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 127, 0, 127);
  for (int g = 0; g < 16; ++g) C[((g & 3) + 8 * (g >> 2) + 4 * h) * 32 + r] = c[g];
}

static float e2m1(unsigned c) {
  const float mag[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
  return (c & 8) ? -mag[c & 7] : mag[c & 7];
}

int main() {
  unsigned char hA[2048], hB[2048];
  float hC[1024], ref[1024];
  srand(7);
  for (int i = 0; i < 2048; ++i) { hA[i] = rand() & 15; hB[i] = rand() & 15; }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      double s = 0;
      for (int kk = 0; kk < 64; ++kk) s += (double)e2m1(hA[i * 64 + kk]) * e2m1(hB[kk * 32 + j]);
      ref[i * 32 + j] = (float)s;
    }
  unsigned char *dA, *dB; float* dC;
  (void)hipMalloc(&dA, 2048); (void)hipMalloc(&dB, 2048); (void)hipMalloc(&dC, 4096);
  (void)hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
  int bad[2];
  for (int hf = 0; hf < 2; ++hf) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC, hf);
    (void)hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
    bad[hf] = 0;
    for (int i = 0; i < 1024; ++i) bad[hf] += hC[i] != ref[i];
  }
  printf("{\"mfma_scale_32x32x64_fp4_mismatches_lo_first\": %d, \"hi_first\": %d, \"sample\": [%g, %g]}\n",
         bad[0], bad[1], hC[0], ref[0]);
  return 0;
}
