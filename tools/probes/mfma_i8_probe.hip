// Verifies the lane maps assumed by the MFMA Hamming kernel for v_mfma_i32_32x32x32_i8:
//   A: lane l, byte j -> A[l&31][16*(l>>5)+j];  B: lane l, byte j -> B[16*(l>>5)+j][l&31]
//   C: lane l, reg r  -> C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__global__ void k(const signed char* A, const signed char* B, int* C) {
  const int l = threadIdx.x, h = l >> 5, r = l & 31;
  v4i a, b;
  signed char* pa = (signed char*)&a;
  signed char* pb = (signed char*)&b;
  for (int j = 0; j < 16; ++j) {
    pa[j] = A[r * 32 + 16 * h + j];
    pb[j] = B[(16 * h + j) * 32 + r];
  }
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
  for (int g = 0; g < 16; ++g) C[((g & 3) + 8 * (g >> 2) + 4 * h) * 32 + r] = c[g];
}

int main() {
  signed char hA[1024], hB[1024];
  int hC[1024], ref[1024];
  srand(7);
  for (int i = 0; i < 1024; ++i) { hA[i] = (signed char)(rand() % 7 - 3); hB[i] = (signed char)(rand() % 5 - 2); }
  for (int i = 0; i < 32; ++i)
    for (int j = 0; j < 32; ++j) {
      int s = 0;
      for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[kk * 32 + j];
      ref[i * 32 + j] = s;
    }
  signed char *dA, *dB; int* dC;
  (void)hipMalloc(&dA, 1024); (void)hipMalloc(&dB, 1024); (void)hipMalloc(&dC, 4096);
  (void)hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  (void)hipMemcpy(hC, dC, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 1024; ++i) bad += hC[i] != ref[i];
  printf("{\"mfma_i32_32x32x32_i8_layout_mismatches\": %d}\n", bad);
  return bad != 0;
}
