// mfma_common.h -- device helpers shared by the matrix-core kernels (hamming_mfma.hip,
// gemm_topk.hip): compile-time loops, raw barriers / counted waits, and inline-asm LDS accesses
// that the compiler cannot tie to an outstanding LDS-DMA (see the note below).
#pragma once

#include <type_traits>

#include "vrq_internal.h"

namespace vrq {

typedef int v2i __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v4f __attribute__((ext_vector_type(4)));

// compile-time loop: f(integral_constant<int, I>) for I in [I0, N) -- every index a constant,
// so register arrays indexed by it stay in registers (a #pragma unroll may give up)
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

__device__ __forceinline__ void barrier_all() { asm volatile("s_barrier" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// LDS accesses inside the tile loop are inline asm: after a global_load_lds the compiler
// would otherwise put s_waitcnt vmcnt(0) before the next LDS access (it cannot tell the
// DMA's target apart), stalling every tile on the DMA just issued.  Loaded registers become
// valid at the matching wait, which takes them as "+v" operands so no use is hoisted above it.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void*)p);
}
__device__ __forceinline__ void lds_read128(v4i& d, uint32_t a) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(d) : "v"(a) : "memory");
}
// the same read into a loop-carried register set: the destination is an in/out operand, so the read,
// its wait and the loop-carried value form one tied chain the register allocator keeps in one place
// (an output-only destination may be given other registers and copied into the carried ones before
// the wait retires the load -- tests/isa_check.py)
__device__ __forceinline__ void lds_read128_inplace(v4i& d, uint32_t a) {
  asm volatile("ds_read_b128 %0, %1" : "+v"(d) : "v"(a) : "memory");
}
template <int OFF>
__device__ __forceinline__ void lds_read128_imm(v4i& d, uint32_t a) {  // address + immediate offset
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}
__device__ __forceinline__ void lds_read64(v2i& d, uint32_t a) {
  asm volatile("ds_read_b64 %0, %1" : "=v"(d) : "v"(a) : "memory");
}
__device__ __forceinline__ void lds_read32(int& d, uint32_t a) {
  asm volatile("ds_read_b32 %0, %1" : "=v"(d) : "v"(a) : "memory");
}
__device__ __forceinline__ void lds_read32_inplace(int& d, uint32_t a) {
  asm volatile("ds_read_b32 %0, %1" : "+v"(d) : "v"(a) : "memory");
}
__device__ __forceinline__ void lds_write128(uint32_t a, const v4i& v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_write32(uint32_t a, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_add32(uint32_t a, int v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_add_rtn32(int& d, uint32_t a, int v) {
  asm volatile("ds_add_rtn_u32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(v) : "memory");
}
#define VRQ_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

}  // namespace vrq
