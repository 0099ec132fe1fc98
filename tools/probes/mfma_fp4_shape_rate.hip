// Rate probe: does the FP4 MFMA shape change the clock the chip holds under the lean K1r loop's work?
// (Timing only; not product code.)  Per wave 64 queries, per 32-row n-block 1024 dims, B unpacked from
// packed 32-bit row words by the scan's 5-VALU unpack, two waves per SIMD (8 per CU), random bits:
//   S32: v_mfma_scale_f32_32x32x64_f8f6f4, 16 k-steps x 2 query blocks of 32 per n-block (shipped)
//   S16: v_mfma_scale_f32_16x16x128_f8f6f4, 8 k-steps x 2 row blocks x 4 query blocks of 16
// Same MFMA work and the same unpack VALU per n-block; row words from LDS (ds_read_b128, as K1r).
// Prints wall time, TOPS and the in-kernel clock (s_memtime / s_memrealtime) per shape, alternated.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v4i unpack_row32(uint32_t w) {
  v4i r;
  r.x = (int)(w & 0x11111111u);
  r.y = (int)(w & 0x22222222u);
  r.z = (int)(w & 0x44444444u);
  r.w = (int)((w >> 1) & 0x44444444u);
  return r;
}

template <int S>
__global__ __launch_bounds__(512, 1) void probe(const v4i* __restrict__ src, int iters, float* __restrict__ out,
                                                unsigned long long* __restrict__ clk) {
  __shared__ v4i tile[4096];  // 64 KiB of packed rows
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4096; i += 512) tile[i] = src[(blockIdx.x * 4096 + i) & 65535];
  __syncthreads();
  v4i A[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) A[s] = src[(w * 2048 + s * 64 + l) & 65535] & 0x11111111;
#pragma unroll
  for (int s = 0; s < 32; ++s) asm volatile("" : "+a"(A[s]));
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  v16f acc32[2] = {};
  v4f acc16[8] = {};
  const uint32_t base = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void*)&tile[0]) +
                        (uint32_t)((w * 64 + l) * 64);
  for (int it = 0; it < iters; ++it) {
    const uint32_t tb = base + (uint32_t)((it & 1) * 32768);
    v4i rb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(rb[q]) : "v"(tb), "n"(q * 16));
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rb[0]), "+v"(rb[1]), "+v"(rb[2]), "+v"(rb[3]));
    if constexpr (S == 32) {
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const v4i b = unpack_row32((uint32_t)rb[s >> 2][s & 3]);
        const v8i b8 = {b.x, b.y, b.z, b.w, 0, 0, 0, 0};
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const v4i a = A[2 * s + m];
          const v8i a8 = {a.x, a.y, a.z, a.w, 0, 0, 0, 0};
          acc32[m] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc32[m], 4, 4, 0, 0, 0, 0);
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
          const v4i b = unpack_row32((uint32_t)rb[(2 * s + nb) >> 2][(2 * s + nb) & 3]);
          const v8i b8 = {b.x, b.y, b.z, b.w, 0, 0, 0, 0};
#pragma unroll
          for (int m = 0; m < 4; ++m) {
            const v4i a = A[4 * s + m];
            const v8i a8 = {a.x, a.y, a.z, a.w, 0, 0, 0, 0};
            acc16[2 * m + nb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a8, b8, acc16[2 * m + nb], 4, 4, 0, 0, 0, 0);
          }
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float sum = 0.f;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int g = 0; g < 16; ++g) sum += acc32[m][g];
#pragma unroll
  for (int b = 0; b < 8; ++b) sum += acc16[b].x + acc16[b].y + acc16[b].z + acc16[b].w;
  out[blockIdx.x * 512 + threadIdx.x] = sum;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200000;
  const int grid = 256;
  v4i* src;
  float* out;
  unsigned long long* clk;
  (void)hipMalloc(&src, 65536 * 16);
  (void)hipMalloc(&out, grid * 512 * 4);
  (void)hipMalloc(&clk, grid * 16);
  int* h = (int*)malloc(65536 * 16);
  srand(11);
  for (int i = 0; i < 65536 * 4; ++i) h[i] = rand() ^ (rand() << 16);
  (void)hipMemcpy(src, h, 65536 * 16, hipMemcpyHostToDevice);
  unsigned long long hc[512];
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 6; ++rep) {
    const int s = rep & 1 ? 16 : 32;
    (void)hipEventRecord(e0, 0);
    if (s == 32)
      hipLaunchKernelGGL(probe<32>, dim3(grid), dim3(512), 0, 0, src, iters, out, clk);
    else
      hipLaunchKernelGGL(probe<16>, dim3(grid), dim3(512), 0, 0, src, iters, out, clk);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(hc, clk, grid * 16, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int b = 0; b < grid; ++b) ghz += (double)hc[2 * b] / ((double)hc[2 * b + 1] * 10.0);
    ghz /= grid;
    const double ops = (double)grid * 8 * iters * 64.0 * 32.0 * 1024.0 * 2.0;  // 64 queries x 32 rows x 1024 dims
    printf("{\"shape\": %d, \"iters\": %d, \"ms\": %.3f, \"TOPS\": %.1f, \"clock_ghz\": %.3f}\n", s, iters, ms,
           ops / (ms * 1e-3) / 1e12, ghz);
  }
  return 0;
}
