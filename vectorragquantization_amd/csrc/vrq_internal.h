// vrq_internal.h -- shared device helpers for the gfx950 kernels of libvrq.so.
// Written for CDNA4 wave64 only (no CUDA/HIP dual paths).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vrq.h"

namespace vrq {

constexpr int WAVE = 64;
constexpr uint64_t KEY_NONE = ~0ull;   // sentinel (dist = INF, row = max)
constexpr int KEY_ROW_BITS = 40;       // global candidate key: dist << 40 | row
constexpr int32_t DIST_NONE = 0x7fffffff;

#define VRQ_CHECK_ARG(c)            \
  do {                              \
    if (!(c)) return VRQ_EINVAL;    \
  } while (0)

#define VRQ_LAUNCH_CHECK()                               \
  do {                                                   \
    if (hipPeekAtLastError() != hipSuccess) {            \
      (void)hipGetLastError();                           \
      return VRQ_EHIP;                                   \
    }                                                    \
  } while (0)

// Planning overrides for sweeps.  Only the probe build (libvrq_probe.so, compiled with
// -DVRQ_TUNING_ENV for tools/ and one test) reads them from the environment; the release
// libvrq.so always plans with the defaults, whatever the environment holds.
#ifdef VRQ_TUNING_ENV
}  // namespace vrq
#include <stdlib.h>
namespace vrq {
inline int tuning_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e && *e ? atoi(e) : dflt;
}
#else
inline int tuning_int(const char*, int dflt) { return dflt; }
#endif

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t shfl_xor_u32(uint32_t v, int m) {
  return (uint32_t)__shfl_xor((int)v, m, WAVE);
}

// Wave butterflies without the LDS crossbar.  A __shfl_xor is a ds_bpermute round trip (~100+ cycles
// on the wave's critical path, twice for 64-bit values); here lane l meets lane l ^ M through
//   M = 1, 2: quad_perm DPP;
//   M = 4, 8: the half-row / row mirror DPP, which pair lane l with a lane of the group l ^ M -- the
//             same value once every group of M lanes holds a single value, which the steps below M
//             establish for a commutative combine;
//   M = 16, 32: v_permlane16/32_swap, which hand every lane both values of its pair.
// Each lane then computes OP(own, partner) or OP(partner, own); for a commutative OP that is the
// value the __shfl_xor butterfly computes, bit for bit.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
template <int M>
__device__ __forceinline__ uint32_t dpp_partner_u32(uint32_t x) {
  static_assert(M == 1 || M == 2 || M == 4 || M == 8, "DPP butterfly step");
  return dpp_u32<M == 1 ? 0xB1 : M == 2 ? 0x4E : M == 4 ? 0x141 : 0x140>(x);
}
// one butterfly step on a 64-bit value (T = double / int64_t), combined by OP
template <int M, class T, class OP>
__device__ __forceinline__ T bfly64(T v, OP op) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)u, hi = (uint32_t)(u >> 32);
  if constexpr (M <= 8) {
    const uint64_t p = ((uint64_t)dpp_partner_u32<M>(hi) << 32) | dpp_partner_u32<M>(lo);
    return op(v, __builtin_bit_cast(T, p));
  } else {
    const auto pl = M == 16 ? __builtin_amdgcn_permlane16_swap(lo, lo, false, false)
                            : __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = M == 16 ? __builtin_amdgcn_permlane16_swap(hi, hi, false, false)
                            : __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const T a = __builtin_bit_cast(T, ((uint64_t)ph[0] << 32) | pl[0]);  // the pair's lower-group value
    const T b = __builtin_bit_cast(T, ((uint64_t)ph[1] << 32) | pl[1]);  // ... and its upper-group value
    return op(a, b);
  }
}
template <class T, class OP>
__device__ __forceinline__ T wave_allreduce64(T v, OP op) {
  v = bfly64<1>(v, op);
  v = bfly64<2>(v, op);
  v = bfly64<4>(v, op);
  v = bfly64<8>(v, op);
  v = bfly64<16>(v, op);
  return bfly64<32>(v, op);
}

// f64 wave sum (butterfly; identical result in every lane)
__device__ __forceinline__ double wave_sum_f64(double v) {
  return wave_allreduce64(v, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
  return wave_allreduce64(v, [](int64_t a, int64_t b) { return a + b; });
}

// Sortable 64-bit image of a double for DESCENDING order: larger double -> smaller key.
// -0.0 maps to the key of +0.0: Python's sort (the reference) treats them as equal.
__device__ __forceinline__ uint64_t desc_key_f64(double x) {
  if (x == 0.0) x = 0.0;
  uint64_t u = (uint64_t)__double_as_longlong(x);
  u = (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);  // ascending image
  return ~u;                                                            // descending
}

// Block-wide (LDS) bitonic sort of n_pow2 u64 keys, ascending.  All threads of the
// block call it; n_pow2 is a power of two <= capacity of `a`.
__device__ inline void block_bitonic_sort_u64(uint64_t* a, int n_pow2) {
  for (int size = 2; size <= n_pow2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < (n_pow2 >> 1); i += blockDim.x) {
        int lo = ((i / stride) * stride * 2) + (i % stride);
        int hi = lo + stride;
        bool up = ((lo & size) == 0);
        uint64_t x = a[lo], y = a[hi];
        if ((x > y) == up) {
          a[lo] = y;
          a[hi] = x;
        }
      }
    }
  }
  __syncthreads();
}

// Same, sorting (key, payload) pairs by key.
__device__ inline void block_bitonic_sort_kv(uint64_t* k, int32_t* v, int n_pow2) {
  for (int size = 2; size <= n_pow2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < (n_pow2 >> 1); i += blockDim.x) {
        int lo = ((i / stride) * stride * 2) + (i % stride);
        int hi = lo + stride;
        bool up = ((lo & size) == 0);
        uint64_t x = k[lo], y = k[hi];
        if ((x > y) == up) {
          k[lo] = y;
          k[hi] = x;
          int32_t t = v[lo];
          v[lo] = v[hi];
          v[hi] = t;
        }
      }
    }
  }
  __syncthreads();
}

__host__ __device__ constexpr int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace vrq
