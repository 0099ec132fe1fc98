// Rate probe for a role-swapped K1m (timing only; not product code): corpus rows stationary as the
// MFMA A operand (RB row blocks of 32 rows x 1024 dims per wave, 64 x RB AGPRs), queries streamed
// from LDS as packed bits (512 queries x 128 B = 64 KiB per workgroup) and unpacked per k-step with
// the 5-VALU row unpack; per 32-query block: 16 k-steps x RB MFMAs (32x32x64 FP4) seeded from
// zero (the seeds' cost is not modelled), then the max3-tree threshold test of the previous block's RB accumulators in
// this block's MFMA shadow, no barrier.  Variants: RB = 4 with one wave per SIMD, RB = 2 with two, each
// with and without a row-set switch every 16 blocks (A rebuilt from LDS: 7-VALU unpack + AGPR writes).
// Prints TOPS and the in-kernel clock.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ v4i unpack_row32(uint32_t w) {
  v4i r;
  r.x = (int)(w & 0x11111111u);
  r.y = (int)(w & 0x22222222u);
  r.z = (int)(w & 0x44444444u);
  r.w = (int)((w >> 1) & 0x44444444u);
  return r;
}
__device__ __forceinline__ v16f mfma(const v4i& a, const v4i& b, const v16f& c) {
  const v8i a8 = {a.x, a.y, a.z, a.w, 0, 0, 0, 0};
  const v8i b8 = {b.x, b.y, b.z, b.w, 0, 0, 0, 0};
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, 4, 4, 0, 0, 0, 0);
}
__device__ __forceinline__ bool any_above(const v16f& a, float thr) {
  const v16i b = __builtin_bit_cast(v16i, a);
  const int x0 = max(max(b[0], b[1]), b[2]), x1 = max(max(b[3], b[4]), b[5]), x2 = max(max(b[6], b[7]), b[8]);
  const int x3 = max(max(b[9], b[10]), b[11]), x4 = max(max(b[12], b[13]), b[14]);
  return __ballot(max(max(max(x0, x1), x2), max(max(x3, x4), b[15])) > __float_as_int(thr)) != 0;
}

template <int RB, int NW, bool REBUILD>
__global__ __launch_bounds__(NW * 64, 1) void probe(const uint32_t* __restrict__ src, int iters, int* __restrict__ out,
                                                unsigned long long* __restrict__ clk) {
  __shared__ v4i q[16 * 4 * 64];  // [q-block][group of 4 k-steps][lane] 16 B
  __shared__ float thr[512];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;  // (w < NW)
  for (int i = threadIdx.x; i < 16 * 4 * 64; i += NW * 64) {
    const uint32_t* s = src + ((blockIdx.x * 4096 + i * 4) & 262143);
    q[i] = v4i{(int)s[0], (int)s[1], (int)s[2], (int)s[3]};
  }
  for (int i = threadIdx.x; i < 512; i += NW * 64) thr[i] = 300.0f + (float)(src[i] & 255);
  __syncthreads();
  v4i A[RB][16];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const uint32_t x = src[(w * 8192 + (r * 16 + s) * 64 + l) & 262143];
      A[r][s] = v4i{(int)((x << 2) & 0x44444444u), (int)(x & 0x22222222u), (int)((x >> 2) & 0x11111111u),
                    (int)((x >> 3) & 0x11111111u)};
    }
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int s = 0; s < 16; ++s) asm volatile("" : "+a"(A[r][s]));
  v16f seed[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int g = 0; g < 16; ++g) seed[r][g] = -(float)(src[(r * 16 + g + l) & 262143] & 511) * 0.5f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  v16f acc[2][RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) acc[0][r] = acc[1][r] = seed[r];
  int hits = 0;
  for (int it = 0; it < iters; ++it) {
    if (REBUILD) {  // a row-set switch: the next rows' A fragments from LDS (packed) + unpack
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const v4i x = q[((it + r * 4 + g) & 63) * 64 + l];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t wd = (uint32_t)x[j];
            A[r][4 * g + j] = v4i{(int)((wd << 2) & 0x44444444u), (int)(wd & 0x22222222u),
                                  (int)((wd >> 2) & 0x11111111u), (int)((wd >> 3) & 0x11111111u)};
            asm volatile("" : "+a"(A[r][4 * g + j]));
          }
        }
    }
    for (int qp = 0; qp < 8; ++qp) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int qb = 2 * qp + c;
        const float th = thr[qb * 32 + (l & 31)];
        v4i wq[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) wq[g] = q[(qb * 4 + g) * 64 + l];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const v4i b = unpack_row32((uint32_t)wq[s >> 2][s & 3]);
#pragma unroll
          for (int r = 0; r < RB; ++r) acc[c][r] = mfma(A[r][s], b, s == 0 ? v16f{} : acc[c][r]);
          if (s == 4) {
#pragma unroll
            for (int r = 0; r < RB; ++r) hits += any_above(acc[c ^ 1][r], th) ? 1 : 0;
          }
        }
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int g = 0; g < 16; ++g) sum += acc[c][r][g];
  out[blockIdx.x * (NW * 64) + threadIdx.x] = hits + (int)sum + (int)seed[0][0];
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  const int grid = 256;
  uint32_t* src;
  int* out;
  unsigned long long* clk;
  (void)hipMalloc(&src, 262144 * 4);
  (void)hipMalloc(&out, grid * 512 * 4);
  (void)hipMalloc(&clk, grid * 16);
  uint32_t* h = (uint32_t*)malloc(262144 * 4);
  srand(7);
  for (int i = 0; i < 262144; ++i) h[i] = (uint32_t)rand() ^ ((uint32_t)rand() << 16);
  (void)hipMemcpy(src, h, 262144 * 4, hipMemcpyHostToDevice);
  unsigned long long hc[512];
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int rep = 0; rep < 9; ++rep) {
    // 0: RB4 NW4, 1: RB4 NW4 + rebuild, 3: RB2 NW8 + rebuild (RB2 NW8 without the rebuild: the compiler
    // spills it, not timed)
    const int cfg = rep % 3 == 2 ? 3 : rep % 3;
    const int rb = cfg < 2 ? 4 : 2, nw = cfg < 2 ? 4 : 8, rebuild = cfg & 1;
    (void)hipEventRecord(e0, 0);
    if (cfg == 0) hipLaunchKernelGGL((probe<4, 4, false>), dim3(grid), dim3(256), 0, 0, src, iters, out, clk);
    if (cfg == 1) hipLaunchKernelGGL((probe<4, 4, true>), dim3(grid), dim3(256), 0, 0, src, iters, out, clk);
    if (cfg == 3) hipLaunchKernelGGL((probe<2, 8, true>), dim3(grid), dim3(512), 0, 0, src, iters, out, clk);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipMemcpy(hc, clk, grid * 16, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int b = 0; b < grid; ++b) ghz += (double)hc[2 * b] / ((double)hc[2 * b + 1] * 10.0);
    ghz /= grid;
    const double ops = (double)grid * nw * iters * 16.0 * 16.0 * rb * 131072.0;
    printf("{\"row_blocks\": %d, \"waves\": %d, \"rebuild_every_16_qblocks\": %d, \"iters\": %d, \"ms\": %.3f, \"TOPS\": %.1f, \"clock_ghz\": %.3f, \"frac_of_10066\": %.3f}\n",
           rb, nw, rebuild, iters, ms, ops / (ms * 1e-3) / 1e12, ghz, ops / (ms * 1e-3) / 1e12 / 10066.3);
  }
  return 0;
}
