// dequant.hip -- the search side of the VectorDBInt{4,8,16}{,Global} classes: dequantisation of the
// stored codes and the dequantised-dot rescoring of Phase-I candidates.
//
// Reference arithmetic (NumPy 2 scalar rules, reproduced bit for bit):
//   VRQ_ENC_INT8_GLOBAL   VectorDBInt8Global._dequantize_int8  (:144-152)  f32(x) * f32(limit / 127.0)
//   VRQ_ENC_INT16_GLOBAL  VectorDBInt16Global._dequantize_int16 (:144-152) f32(x) * f32(limit / 32767.0)
//   VRQ_ENC_INT4_GLOBAL   VectorDBInt4Global._dequantize_int4  (:166-188)  f32((nib - 8) * (limit / 7.0)), f64 product
//   VRQ_ENC_INT8_LOCAL    VectorDBInt8._dequantize_int8        (:129-138)  0 if min == max, else
//                         f32(x) * (max(|min|, |max|) / 127 in float32: min/max are np.float32)
//   VRQ_ENC_INT4_LOCAL    VectorDBInt4._dequantize_int4        (:157-184)  0 if min == max, else
//                         f32((nib - 8) * (max(|min|, |max|) / 7.0)), f64 (min/max are Python floats)
// Int4 bytes hold element 2i in the high nibble and 2i+1 in the low nibble (value + 8).
// Rescoring (VectorDBInt8Global.py:232-238 and the same loop in the other classes):
//   score = float(np.dot(query_float, dequantised row)), a float32 dot: computed here as the exact
//   f64 sum of the exact f32 x f32 products rounded once to f32 (NumPy's sdot is within a few ulp).
//   VRQ_RESCORE_F32 (rescoring only): the compare_float32 branch (VectorDBInt8Global.py:239-240 and
//   the same branch in the other classes) -- q is the f32 float_embeddings rows, used as they are.
#include "vrq_internal.h"

namespace vrq {

constexpr int DQ_MAX_DIM = 8192;

struct DeqRow {
  int mode;
  double limit;
  float sf;   // float32 scale (INT8/INT16 global, INT8 local)
  double sd;  // float64 scale (INT4 modes)
  bool zero;  // local modes with min == max
};

__device__ __forceinline__ DeqRow deq_row(int mode, double limit, const double* minmax, int64_t r) {
  DeqRow d{mode, limit, 0.f, 0.0, false};
  switch (mode) {
    case VRQ_RESCORE_F32: break;
    case VRQ_ENC_INT8_GLOBAL: d.sf = (float)(limit / 127.0); break;
    case VRQ_ENC_INT16_GLOBAL: d.sf = (float)(limit / 32767.0); break;
    case VRQ_ENC_INT4_GLOBAL: d.sd = limit / 7.0; break;
    case VRQ_ENC_INT8_LOCAL: {
      const float mn = (float)minmax[2 * r], mx = (float)minmax[2 * r + 1];
      d.zero = mn == mx;
      d.sf = __fdiv_rn(fmaxf(fabsf(mn), fabsf(mx)), 127.0f);  // np.float32 / int -> float32
      break;
    }
    default: {  // VRQ_ENC_INT4_LOCAL
      const double mn = minmax[2 * r], mx = minmax[2 * r + 1];
      d.zero = mn == mx;
      d.sd = fmax(fabs(mn), fabs(mx)) / 7.0;
      break;
    }
  }
  return d;
}

// element i of row r (q = the mode's code array)
__device__ __forceinline__ float deq_elem(const DeqRow& d, const void* q, int64_t r, int dim, int i) {
  if (d.zero) return 0.f;
  switch (d.mode) {
    case VRQ_RESCORE_F32:
      return reinterpret_cast<const float*>(q)[r * dim + i];
    case VRQ_ENC_INT8_GLOBAL:
    case VRQ_ENC_INT8_LOCAL:
      return __fmul_rn((float)reinterpret_cast<const int8_t*>(q)[r * dim + i], d.sf);
    case VRQ_ENC_INT16_GLOBAL:
      return __fmul_rn((float)reinterpret_cast<const int16_t*>(q)[r * dim + i], d.sf);
    default: {
      const uint8_t b = reinterpret_cast<const uint8_t*>(q)[r * ((dim + 1) / 2) + (i >> 1)];
      const int nib = (i & 1) ? (b & 15) : (b >> 4);
      return (float)__dmul_rn((double)(nib - 8), d.sd);
    }
  }
}

__global__ __launch_bounds__(256) void dequant_kernel(int mode, const void* __restrict__ q,
                                                      const double* __restrict__ minmax, int64_t n, int dim,
                                                      double limit, float* __restrict__ out) {
  const int64_t r = blockIdx.x;
  if (r >= n) return;
  const DeqRow d = deq_row(mode, limit, minmax, r);
  for (int i = threadIdx.x; i < dim; i += 256) out[r * dim + i] = deq_elem(d, q, r, dim, i);
}

// one wave per (query, candidate); negative candidate rows -> NaN
__global__ __launch_bounds__(256) void rescore_dequant_kernel(int mode, const float* __restrict__ qf, int nq, int dim,
                                                              const void* __restrict__ q,
                                                              const double* __restrict__ minmax, double limit,
                                                              int64_t n, const int64_t* __restrict__ cand,
                                                              int ncand, double* __restrict__ out) {
  const int64_t wv = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = lane_id();
  if (wv >= (int64_t)nq * ncand) return;
  const int qi = (int)(wv / ncand);
  const int64_t r = cand[wv];
  if (r < 0 || r >= n) {
    if (l == 0) out[wv] = __builtin_nan("");
    return;
  }
  const DeqRow d = deq_row(mode, limit, minmax, r);
  double s = 0.0;
  for (int i = l; i < dim; i += WAVE) s += (double)qf[(int64_t)qi * dim + i] * (double)deq_elem(d, q, r, dim, i);
  s = wave_sum_f64(s);  // exact products, f64 accumulation, one rounding to f32 below
  if (l == 0) out[wv] = (double)(float)s;
}

}  // namespace vrq

using namespace vrq;

extern "C" {

int vrq_dequantize(int32_t mode, const void* q, const double* minmax, int64_t n, int32_t dim, double limit,
                   float* out, void* stream) {
  VRQ_CHECK_ARG(mode >= VRQ_ENC_INT8_GLOBAL && mode <= VRQ_ENC_INT4_LOCAL);
  VRQ_CHECK_ARG(n >= 0 && dim > 0);
  if (dim > DQ_MAX_DIM) return VRQ_EUNSUPPORTED;
  if (n == 0) return VRQ_OK;
  VRQ_CHECK_ARG(q && out);
  if (mode == VRQ_ENC_INT8_LOCAL || mode == VRQ_ENC_INT4_LOCAL) VRQ_CHECK_ARG(minmax);
  // one workgroup per row; launches of at most 2^22 rows keep a dispatch below 2^32 work-items
  const int64_t qrow = mode == VRQ_ENC_INT16_GLOBAL                              ? 2 * (int64_t)dim
                       : (mode == VRQ_ENC_INT4_GLOBAL || mode == VRQ_ENC_INT4_LOCAL) ? (int64_t)(dim + 1) / 2
                                                                                    : (int64_t)dim;
  constexpr int64_t kMaxLaunch = 1 << 22;
  for (int64_t r0 = 0; r0 < n; r0 += kMaxLaunch) {
    const int64_t nr = n - r0 < kMaxLaunch ? n - r0 : kMaxLaunch;
    hipLaunchKernelGGL(dequant_kernel, dim3((unsigned)nr), dim3(256), 0, (hipStream_t)stream, (int)mode,
                       (const void*)((const uint8_t*)q + r0 * qrow), minmax ? minmax + 2 * r0 : nullptr, nr, (int)dim,
                       limit, out + r0 * dim);
    VRQ_LAUNCH_CHECK();
  }
  return VRQ_OK;
}

int vrq_rescore_dequant(int32_t mode, const float* qf, int32_t nq, int32_t dim, const void* q, const double* minmax,
                        double limit, int64_t n, const int64_t* cand_rows, int32_t ncand, double* out,
                        void* stream) {
  VRQ_CHECK_ARG((mode >= VRQ_ENC_INT8_GLOBAL && mode <= VRQ_ENC_INT4_LOCAL) || mode == VRQ_RESCORE_F32);
  VRQ_CHECK_ARG(nq >= 0 && ncand >= 0 && n >= 0 && dim > 0);
  if (dim > DQ_MAX_DIM) return VRQ_EUNSUPPORTED;
  if (nq == 0 || ncand == 0) return VRQ_OK;
  VRQ_CHECK_ARG(qf && q && cand_rows && out);
  if (mode == VRQ_ENC_INT8_LOCAL || mode == VRQ_ENC_INT4_LOCAL) VRQ_CHECK_ARG(minmax);
  const int64_t waves = (int64_t)nq * ncand;
  hipLaunchKernelGGL(rescore_dequant_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
                     (int)mode, qf, (int)nq, (int)dim, q, minmax, limit, n, cand_rows, (int)ncand, out);
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

}  // extern "C"
