// Raw issue rate of the MFMA forms used by the Phase-I kernels: 4 independent accumulator
// chains per wave, operands in registers, one wave per SIMD over the whole chip (256 CUs x 4).
// Prints cycles per instruction per SIMD (from the wall time at the measured clock-independent
// rate) and the achieved dense ops/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

template <int KIND>
__global__ __launch_bounds__(256) void k(int iters, float* out, int seed) {
  const int l = threadIdx.x;
  v8i a = {l ^ seed, l * 3, l + 7, l * 5, 0, 0, 0, 0}, b = {l * 11, l ^ 9, l + 1, l * 13, 0, 0, 0, 0};
  v16f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  v16i i0 = {0}, i1 = {0}, i2 = {0}, i3 = {0};
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, 4, 4, 0, 128, 0, 128);
      c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c1, 4, 4, 0, 128, 0, 128);
      c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c2, 4, 4, 0, 128, 0, 128);
      c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c3, 4, 4, 0, 128, 0, 128);
    } else {
      const v4i a4 = {a[0], a[1], a[2], a[3]}, b4 = {b[0], b[1], b[2], b[3]};
      i0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, i0, 0, 0, 0);
      i1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, i1, 0, 0, 0);
      i2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, i2, 0, 0, 0);
      i3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, i3, 0, 0, 0);
    }
  }
  long long t1 = clock64();
  float s = 0;
  for (int g = 0; g < 16; ++g) s += c0[g] + c1[g] + c2[g] + c3[g] + (float)(i0[g] + i1[g] + i2[g] + i3[g]);
  out[blockIdx.x * 256 + l] = s;
  if (blockIdx.x == 0 && l == 0) out[1 << 20] = (float)(t1 - t0);
}

int main() {
  float* out;
  (void)hipMalloc(&out, (1 << 20) * 4 + 64);
  const int iters = 20000;
  const char* names[2] = {"mfma_scale_f32_32x32x64_fp4", "mfma_i32_32x32x32_i8"};
  for (int kind = 0; kind < 2; ++kind) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0, 0);
      if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, iters, out, rep);
      else hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, iters, out, rep);
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
    }
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    float cyc;
    (void)hipMemcpy(&cyc, out + (1 << 20), 4, hipMemcpyDeviceToHost);
    const double insts = 4.0 * iters;                       // per wave
    const double ops_per_inst = kind == 0 ? 32.0 * 32 * 64 * 2 : 32.0 * 32 * 32 * 2;
    const double total = insts * 1024 * ops_per_inst;        // 1024 waves
    printf("{\"%s\": {\"ms\": %.3f, \"clock64_cycles_per_inst\": %.2f, \"TOPS\": %.0f, \"implied_GHz_at_32cyc\": %.3f}}\n",
           names[kind], ms, cyc / insts, total / (ms * 1e-3) / 1e12, insts * 32 / (ms * 1e-3) / 1e9);
  }
  return 0;
}
