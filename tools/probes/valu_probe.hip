// Throughput probe: cycles per wave64 instruction for v_xor_b32, v_bcnt_u32_b32, v_add_u32,
// v_bitop3_b32, v_dot4 when the SIMD is saturated (many independent chains, 8 waves/SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define REP 256
template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t seed) {
  uint32_t a0 = seed ^ threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
  uint32_t k = seed * 0x9e3779b9u;
  for (int i = 0; i < REP; ++i) {
#define STEP(x)                                                                        \
  if (OP == 0) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "s"(k));                \
  if (OP == 1) asm volatile("v_bcnt_u32_b32 %0, %0, %0" : "+v"(x));                    \
  if (OP == 2) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x) : "s"(k));                \
  if (OP == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %0 bitop3:0x96" : "+v"(x) : "s"(k)); \
  if (OP == 4) asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(x) : "s"(k));
    STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

template <int OP>
double run(uint32_t* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int blocks = 256 * 8;  // 8 blocks of 256 threads per CU = 8 waves/SIMD
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, d, (uint32_t)r);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  const double insts = 10.0 * blocks * 4 /*waves*/ * REP * 8;   // wave instructions
  const double simd_cycles = ms * 1e-3 * 2.4e9 * 1024;            // at 2.4 GHz
  return simd_cycles / insts;
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 256 * 8 * 256 * 4 * 4);
  printf("{\"cycles_per_wave_instr_at_2.4GHz\": {\"v_xor_b32\": %.2f, \"v_bcnt_u32_b32\": %.2f, \"v_add_u32\": %.2f, \"v_bitop3_b32\": %.2f, \"v_xad_u32\": %.2f}}\n",
         run<0>(d), run<1>(d), run<2>(d), run<3>(d), run<4>(d));
  return 0;
}
