// Rate probe: does the int8 MFMA shape change the clock the chip holds under K5's load?  (Timing
// only; not product code.)  Both kernels do K5's Phase-III tile work per wave: 32 queries x 32 corpus
// rows x 1024 dims of int8 per tile, A (the queries) resident in AGPRs, B (the rows) re-read from a
// 32 KiB LDS tile by one ds_read_b128 per 1 KiB fragment, two waves per SIMD (8 per CU), random data:
//   S32: v_mfma_i32_32x32x32_i8, 32 k-steps x 1 MFMA per tile (the shipped K5 shape)
//   S16: v_mfma_i32_16x16x64_i8, 16 k-steps x (2 query blocks x 2 row blocks) MFMAs per tile
// Same MFMA work, same LDS bytes, same register footprint.  Prints wall time, TOPS and the in-kernel
// clock (s_memtime / s_memrealtime, 100 MHz) per shape, alternating the shapes.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int S>
__global__ __launch_bounds__(512, 1) void probe(const v4i* __restrict__ src, int iters, int* __restrict__ out,
                                                unsigned long long* __restrict__ clk) {
  __shared__ v4i tile[2][2048];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4096; i += 512) (&tile[0][0])[i] = src[(blockIdx.x * 4096 + i) & 65535];
  __syncthreads();
  v4i A[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) A[s] = src[(w * 2048 + s * 64 + l) & 65535];
#pragma unroll
  for (int s = 0; s < 32; ++s) asm volatile("" : "+a"(A[s]));
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  v16i acc32 = {};
  v4i acc16[4] = {};
  const uint32_t base = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void*)&tile[0][0]) + (uint32_t)(l * 16);
  for (int it = 0; it < iters; ++it) {
    const uint32_t tb = base + (uint32_t)((it & 1) * 32768);
    v4i ring[4];
#pragma unroll
    for (int g = 0; g < 2; ++g) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[g]) : "v"(tb), "n"(g * 1024));
#pragma unroll
    for (int s = 0; s < 32; ++s) {
      if (s + 2 < 32)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(ring[(s + 2) & 3]) : "v"(tb), "n"((s + 2) * 1024));
      asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(ring[s & 3]) : "n"(s + 2 < 32 ? 2 : 31 - s));
      if constexpr (S == 32) {
        acc32 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[s], ring[s & 3], acc32, 0, 0, 0);
      } else {
        // fragment s = k-step s >> 1, row block s & 1; both query blocks (A[s] for block 0, A[s ^ 1] for 1)
        acc16[(s & 1)] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[s], ring[s & 3], acc16[s & 1], 0, 0, 0);
        acc16[2 + (s & 1)] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[s ^ 1], ring[s & 3], acc16[2 + (s & 1)], 0, 0, 0);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  int sum = 0;
  if constexpr (S == 32) {
#pragma unroll
    for (int g = 0; g < 16; ++g) sum += acc32[g];
  } else {
#pragma unroll
    for (int b = 0; b < 4; ++b) sum += acc16[b].x + acc16[b].y + acc16[b].z + acc16[b].w;
  }
  out[blockIdx.x * 512 + threadIdx.x] = sum;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 100000;
  const int grid = 256;
  v4i* src;
  int* out;
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
    const double ops = (double)grid * 8 * iters * 32.0 * 32.0 * 1024.0 * 2.0;
    printf("{\"shape\": %d, \"iters\": %d, \"ms\": %.3f, \"TOPS\": %.1f, \"clock_ghz\": %.3f}\n", s, iters, ms,
           ops / (ms * 1e-3) / 1e12, ghz);
  }
  return 0;
}
