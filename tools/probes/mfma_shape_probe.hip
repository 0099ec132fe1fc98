// MFMA shape / form probe for the FP4 Phase-I scan (hamming_mfma.hip): sustained chip-wide rate of
//   0: v_mfma_scale_f32_32x32x64_f8f6f4 (scales 2^1)     1: v_mfma_f32_32x32x64_f8f6f4 (unscaled)
//   2: v_mfma_scale_f32_16x16x128_f8f6f4 (scales 2^1)    3: v_mfma_f32_16x16x128_f8f6f4 (unscaled)
// on (a) random operands and (b) operands shaped like the scan's (each nibble 0x0 or 0x1 =
// e2m1 0 / 0.5 from random bits), 4 independent accumulator chains per wave, one wave per SIMD on
// every CU; plus a correctness check that the unscaled form adds exactly 0.25 per common set bit.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ uint32_t hsh(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
  return x;
}

template <int KIND, int SPARSE>
__global__ __launch_bounds__(256) void k(int iters, float* out, int seed) {
  const int l = threadIdx.x;
  v8i a, b;
  for (int i = 0; i < 8; ++i) {
    uint32_t x = hsh(l * 977 + i * 131 + seed * 7919 + blockIdx.x), y = hsh(x + 12345);
    if (SPARSE) { x &= 0x11111111u; y &= 0x11111111u; }
    a[i] = i < 4 ? (int)x : 0;
    b[i] = i < 4 ? (int)y : 0;
  }
  v16f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  v4f d0 = {0}, d1 = {0}, d2 = {0}, d3 = {0}, d4 = {0}, d5 = {0}, d6 = {0}, d7 = {0};
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 4, 4, 0, 128, 0, 128);
      c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c1, 4, 4, 0, 128, 0, 128);
      c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c2, 4, 4, 0, 128, 0, 128);
      c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c3, 4, 4, 0, 128, 0, 128);
    } else if (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 4, 4, 0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c1, 4, 4, 0, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c2, 4, 4, 0, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c3, 4, 4, 0, 0, 0, 0);
    } else if (KIND == 2) {  // 2 MFMAs of 16x16x128 = the work of one 32x32x64
#define S16(d) d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d, 4, 4, 0, 128, 0, 128)
      S16(d0); S16(d1); S16(d2); S16(d3); S16(d4); S16(d5); S16(d6); S16(d7);
    } else {
#define U16(d) d = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, d, 4, 4, 0, 0, 0, 0)
      U16(d0); U16(d1); U16(d2); U16(d3); U16(d4); U16(d5); U16(d6); U16(d7);
    }
  }
  long long t1 = clock64();
  float s = 0;
  for (int g = 0; g < 16; ++g) s += c0[g] + c1[g] + c2[g] + c3[g];
  for (int g = 0; g < 4; ++g) s += d0[g] + d1[g] + d2[g] + d3[g] + d4[g] + d5[g] + d6[g] + d7[g];
  out[blockIdx.x * 256 + l] = s;
  if (blockIdx.x == 0 && l == 0) out[1 << 20] = (float)(t1 - t0);
}

// unscaled 32x32x64 on one wave: A = B = one lane pattern; result vs 0.25 * popcount dot
__global__ void check(float* out) {
  const int l = threadIdx.x;
  v8i a = {0}, b = {0};
  for (int i = 0; i < 4; ++i) {
    a[i] = (int)(hsh(l * 17 + i) & 0x11111111u);
    b[i] = (int)(hsh(l * 29 + i + 1000) & 0x11111111u);
  }
  v16f c = {0};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 4, 4, 0, 0, 0, 0);
  v16f e = {0};
  e = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, e, 4, 4, 0, 128, 0, 128);
  for (int g = 0; g < 16; ++g) {
    out[l * 32 + g] = c[g];
    out[l * 32 + 16 + g] = e[g];
  }
}

template <int KIND, int SP>
static void run(const char* name, float* out) {
  const int iters = 20000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k<KIND, SP>), dim3(256), dim3(256), 0, 0, iters, out, rep);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
  }
  float ms, cyc;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipMemcpy(&cyc, out + (1 << 20), 4, hipMemcpyDeviceToHost);
  const double ops = 4.0 * iters * 1024 * (32.0 * 32 * 64 * 2);  // 4 x 32x32x64-equivalents per iter per wave
  printf("{\"form\": \"%s\", \"operands\": \"%s\", \"ms\": %.3f, \"clock64_per_32x32x64_equiv\": %.2f, \"TOPS\": %.0f}\n",
         name, SP ? "0/1 nibbles" : "random", ms, cyc / (4.0 * iters), ops / (ms * 1e-3) / 1e12);
}

int main() {
  float* out;
  (void)hipMalloc(&out, (1 << 20) * 4 + 64);
  hipLaunchKernelGGL(check, dim3(1), dim3(64), 0, 0, out);
  float h[64 * 32];
  (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  int ratio_ok = 1;
  for (int i = 0; i < 64; ++i)
    for (int g = 0; g < 16; ++g)
      if (h[i * 32 + g] * 4.0f != h[i * 32 + 16 + g]) ratio_ok = 0;
  printf("{\"unscaled_is_quarter_of_scaled\": %d, \"sample\": [%g, %g]}\n", ratio_ok, h[0], h[16]);
  run<0, 0>("scale_32x32x64", out);
  run<0, 1>("scale_32x32x64", out);
  run<1, 0>("unscaled_32x32x64", out);
  run<1, 1>("unscaled_32x32x64", out);
  run<2, 0>("scale_16x16x128", out);
  run<2, 1>("scale_16x16x128", out);
  run<3, 0>("unscaled_16x16x128", out);
  run<3, 1>("unscaled_16x16x128", out);
  return 0;
}
