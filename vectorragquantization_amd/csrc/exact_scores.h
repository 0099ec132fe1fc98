// exact_scores.h -- the reference's Phase-II / Phase-III scores of ONE row for one query, one
// wave per (query, row), shared by the fused search finish (select_rescore.hip) and the
// exhaustive matrix-core scorer (gemm_topk.hip), so both produce bit-identical scores.
//   Phase II  (CohereEnhancedVectorDB.py:283-293): float(q . (2*unpackbits(code)-1)), float64
//   Phase III (CohereEnhancedVectorDB.py:302-318): float32(q . int8) / ||int8||, -inf if 0
#pragma once

#include "vrq_internal.h"

namespace vrq {

constexpr int DIM = 1024;        // embedding dim of the fused kernels
constexpr int DPL = DIM / WAVE;  // dims per lane (16)

// Each score is split into the lane's load of the row (phase*_load: the caller may keep several
// rows' loads in flight) and the arithmetic on the loaded slice (phase*_from); phase2_dot /
// phase3_cos / flat_ip are the two in sequence.

// Phase II: this lane's code bytes 2l, 2l+1 (dims 16l..16l+15)
__device__ __forceinline__ uint16_t phase2_load(const uint8_t* __restrict__ code_row) {
  return *reinterpret_cast<const uint16_t*>(code_row + 2 * lane_id());
}
// Phase II score of one code row for the lane-resident query slice (dims 16l..16l+15).
__device__ __forceinline__ double phase2_from(const float (&qv)[DPL], uint16_t b) {
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    // packbits is MSB-first: dim 16l+i lives in byte 2l + i/8 at bit 7 - i%8
    const int bit = (i < 8) ? ((b >> (7 - i)) & 1) : ((b >> (8 + 15 - i)) & 1);
    s += bit ? (double)qv[i] : -(double)qv[i];
  }
  return wave_sum_f64(s);
}
__device__ __forceinline__ double phase2_dot(const float (&qv)[DPL], const uint8_t* __restrict__ code_row) {
  return phase2_from(qv, phase2_load(code_row));
}

// Phase III: this lane's 16 int8 values of the row
__device__ __forceinline__ int4 phase3_load(const int8_t* __restrict__ xrow) {
  return *reinterpret_cast<const int4*>(xrow + DPL * lane_id());
}
// Phase III: float32(q . int8 row) / norm, -inf if norm == 0.
__device__ __forceinline__ double phase3_from(const float (&qv)[DPL], const int4 raw, double nrm) {
  const int32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const int8_t x = (int8_t)((w[i >> 2] >> (8 * (i & 3))) & 0xff);
    s += (double)qv[i] * (double)x;  // exact product
  }
  s = wave_sum_f64(s);                // exact sum
  const float f = (float)s;           // one rounding: correctly rounded float32 dot
  return nrm == 0.0 ? -__builtin_inf() : (double)f / nrm;
}
__device__ __forceinline__ double phase3_cos(const float (&qv)[DPL], const int8_t* __restrict__ xrow, double nrm) {
  return phase3_from(qv, phase3_load(xrow), nrm);
}

// IndexFlatIP (CohereVectorDBFloat.py:62,156): the float32 inner product q . x, computed as the
// exact products summed in float64 and rounded once to float32 (FAISS's sgemm / fvec_inner_product
// round at every step; this is the same value within the float32 summation error).
struct FlatSlice {
  float4 v[DPL / 4];
};
__device__ __forceinline__ FlatSlice flat_load(const float* __restrict__ xrow) {
  const float4* p = reinterpret_cast<const float4*>(xrow + DPL * lane_id());
  FlatSlice x;
#pragma unroll
  for (int i = 0; i < DPL / 4; ++i) x.v[i] = p[i];
  return x;
}
__device__ __forceinline__ double flat_from(const float (&qv)[DPL], const FlatSlice& x) {
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < DPL / 4; ++i) {
    const float4 v = x.v[i];
    s += (double)qv[4 * i + 0] * (double)v.x;
    s += (double)qv[4 * i + 1] * (double)v.y;
    s += (double)qv[4 * i + 2] * (double)v.z;
    s += (double)qv[4 * i + 3] * (double)v.w;
  }
  return (double)(float)wave_sum_f64(s);
}
__device__ __forceinline__ double flat_ip(const float (&qv)[DPL], const float* __restrict__ xrow) {
  return flat_from(qv, flat_load(xrow));
}

// Phase II by nibble tables (one row per thread): tab[p * 16 + v] = sum over the 4 dims 4p .. 4p+3 of
// nibble p (packbits MSB first) of (bit of v ? q : -q), in float64 -- exact, as every partial sum of the
// reference's float32 x +-1 products is -- so the 256-term sum over a code's nibbles is the same exact
// value as phase2_dot.  phase2_table fills the 32 KiB table with a block's `nthreads` threads.
__device__ __forceinline__ void phase2_table(const float* __restrict__ q, double* tab, int tid, int nthreads) {
  for (int e = tid; e < 256 * 16; e += nthreads) {
    const int p = e >> 4, v = e & 15;
    double t = 0.0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const double x = (double)q[4 * p + b];
      t += ((v >> (3 - b)) & 1) ? x : -x;
    }
    tab[e] = t;
  }
}
__device__ __forceinline__ double phase2_nibbles(const double* tab, const uint8_t* __restrict__ code_row) {
  const uint4* src = reinterpret_cast<const uint4*>(code_row);
  uint4 cw[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) cw[i] = src[i];
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t wd[4] = {cw[i].x, cw[i].y, cw[i].z, cw[i].w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int c = 0; c < 4; ++c) {  // byte 16 i + 4 k + c (little-endian in the dword): nibbles 2b, 2b + 1
        const uint32_t byte = (wd[k] >> (8 * c)) & 0xffu;
        const int pb = 2 * (16 * i + 4 * k + c);
        s += tab[pb * 16 + (byte >> 4)];
        s += tab[(pb + 1) * 16 + (byte & 15)];
      }
  }
  return s;
}

__device__ __forceinline__ void load_q(float (&qv)[DPL], const float* __restrict__ q) {
  const int l = lane_id();
  const float4* p = reinterpret_cast<const float4*>(q + DPL * l);
#pragma unroll
  for (int i = 0; i < DPL / 4; ++i) {
    const float4 v = p[i];
    qv[4 * i + 0] = v.x;
    qv[4 * i + 1] = v.y;
    qv[4 * i + 2] = v.z;
    qv[4 * i + 3] = v.w;
  }
}

}  // namespace vrq
