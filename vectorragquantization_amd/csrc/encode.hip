// encode.hip -- K6: the VectorDBInt{4,8,16}{,Global} scalar-quantise + packbits
// encode path, and K7: float64 int8 row norms.  One wave per vector.
//
// Bit-exactness notes (NumPy 2.x semantics of the reference expressions):
//  * _to_binary: packbits(x > np.mean(x)), MSB first.  np.mean(float32) is NumPy's
//    pairwise summation (8 strided accumulators per <=128-element leaf, fixed
//    combine tree, then / n with one rounding to float32).  The leaf / tree
//    structure depends only on n; the host builds it (PwPlan) and the kernel
//    replays it: 8 lanes per leaf accumulate their column sequentially, a 3-step
//    butterfly reproduces ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), one lane adds the
//    leaf's tail and one lane folds the leaves in the recursion's order.  Built
//    with -ffp-contract=off so no add is fused.
//  * scalar scales are Python floats cast to float32 at the multiply (weak
//    scalars): scale32 = (float)(c / limit) in double, which equals the
//    correctly rounded float32 quotient.  np.round = rintf (half to even);
//    .astype(int8) from float truncates (VectorDBInt8.py:126).
//  * VectorDBInt4Global ignores its limit (reference bug, reproduced).
#include "vrq_internal.h"

namespace vrq {

constexpr int MAX_DIM = 8192;
constexpr int MAX_LEAVES = 128;
constexpr int MAX_OPS = 2 * MAX_LEAVES;

struct PwPlan {
  int nleaves;
  int nops;
  int16_t start[MAX_LEAVES];
  int16_t len[MAX_LEAVES];
  int16_t ops[MAX_OPS];  // postfix: >= 0 push leaf sum, -1 add the top two
  int bal_levels;        // L when the tree is the balanced one over 2^L <= 8 leaves in order, else -1
};

// postfix of the balanced tree over leaves [first, first + 2^L): left, right, add
static void pw_balanced(int first, int L, int16_t* ops, int* k) {
  if (L == 0) {
    ops[(*k)++] = (int16_t)first;
    return;
  }
  pw_balanced(first, L - 1, ops, k);
  pw_balanced(first + (1 << (L - 1)), L - 1, ops, k);
  ops[(*k)++] = -1;
}
static void pw_classify(PwPlan* p) {
  p->bal_levels = -1;
  for (int L = 0; L <= 3; ++L) {
    if (p->nleaves != (1 << L)) continue;
    int16_t ops[16];
    int k = 0;
    pw_balanced(0, L, ops, &k);
    bool same = k == p->nops;
    for (int i = 0; same && i < k; ++i) same = ops[i] == p->ops[i];
    if (same) p->bal_levels = L;
  }
}

static void pw_build(int s, int n, PwPlan* p) {
  if (n <= 128) {
    p->start[p->nleaves] = (int16_t)s;
    p->len[p->nleaves] = (int16_t)n;
    p->ops[p->nops++] = (int16_t)p->nleaves++;
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  pw_build(s, n2, p);
  pw_build(s + n2, n - n2, p);
  p->ops[p->nops++] = -1;
}

// The encoder runs one WAVE per vector, EPB vectors per workgroup (fewer, larger workgroups: with
// one 64-thread workgroup per vector the dispatch of ~1M workgroups bounded the launch), each wave
// on its own LDS slice; LDS is shared only inside a wave, so the wave orders its own accesses.
constexpr int EPB = 1;  // 4 measured ~15 % slower (int8g 1.42 -> 1.65 ms per 2^20 vectors)
// (Padding the LDS image by 8 floats per 128 elements, against the bank pattern of the leaf reads,
// measured 4-11 % slower and is not used.)
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// NumPy pairwise float32 sum of x[0..n) staged in LDS; result valid in all lanes.
__device__ float pairwise_sum_f32(const float* x, const PwPlan& P, float* leafsum) {
  const int l = lane_id(), g = l >> 3, j = l & 7;
  float lastres = 0.f;  // lanes 8g: the sum of leaf b + g of the last batch
  for (int b = 0; b < P.nleaves; b += 8) {
    const int li = b + g;
    float r = 0.f;
    int m = 0, s = 0;
    if (li < P.nleaves) {
      s = P.start[li];
      m = P.len[li];
      if (m >= 8) {
        r = x[s + j];
        for (int i = 8; i < m - (m % 8); i += 8) r += x[s + i + j];
      }
    }
    // tree over the 8 accumulators of the leaf (lanes 8g..8g+7)
    float t = r + __shfl_xor(r, 1, WAVE);
    t = t + __shfl_xor(t, 2, WAVE);
    t = t + __shfl_xor(t, 4, WAVE);
    if (j == 0 && li < P.nleaves) {
      float res;
      int i;
      if (m >= 8) {
        res = t;
        i = m - (m % 8);
      } else {
        res = 0.f;
        i = 0;
      }
      for (; i < m; ++i) res += x[s + i];
      leafsum[li] = res;
      lastres = res;
    }
  }
  if (P.bal_levels >= 0) {
    // the balanced tree over <= 8 leaves (dim = 1024: ((L0+L1)+(L2+L3))+((L4+L5)+(L6+L7))), one
    // batch, leaf g in lane 8g: a butterfly over xor 8, 16, 32 performs exactly the tree's additions
    // (float addition is commutative; the association is the tree's)
    float a = lastres;
    if (P.bal_levels >= 1) a = a + __shfl_xor(a, 8, WAVE);
    if (P.bal_levels >= 2) a = a + __shfl_xor(a, 16, WAVE);
    if (P.bal_levels >= 3) a = a + __shfl_xor(a, 32, WAVE);
    return __shfl(a, 0, WAVE);
  }
  wave_lds_sync();
  float out = 0.f;
  if (l == 0) {
    float* st = leafsum + MAX_LEAVES;  // LDS stack (no scratch)
    int sp = 0;
    for (int o = 0; o < P.nops; ++o) {
      const int op = P.ops[o];
      if (op >= 0) {
        st[sp++] = leafsum[op];
      } else {
        const float rgt = st[--sp];
        const float lft = st[--sp];
        st[sp++] = lft + rgt;
      }
    }
    out = st[0];
  }
  return __shfl(out, 0, WAVE);
}

__device__ __forceinline__ float clampf(float v, float lo, float hi) { return fminf(fmaxf(v, lo), hi); }

template <int MODE>
__global__ __launch_bounds__(EPB * 64) void encode_kernel(const void* __restrict__ xin, int64_t n, int dim,
                                                          double limit, uint8_t* __restrict__ codes,
                                                          void* __restrict__ qout, double* __restrict__ minmax,
                                                          PwPlan P, int epb) {
  extern __shared__ __attribute__((aligned(16))) float smem_enc[];
  const int w = threadIdx.x >> 6;
  float* xs = smem_enc + w * (dim + 2 * MAX_LEAVES);  // this wave's dim floats + leaf sums
  float* leafsum = xs + dim;
  const int64_t v = (int64_t)blockIdx.x * epb + w;
  if (v >= n) return;
  const int l = lane_id();
  const int ngroups = dim / 8;
  uint8_t* crow = codes + v * ngroups;

  if constexpr (MODE == VRQ_ENC_BIN_INT16) {
    // VectorDBInt16._to_binary: float64 mean of int16 (exact sum), x > mean
    const int16_t* x = reinterpret_cast<const int16_t*>(xin) + v * dim;
    if (dim == 16 * WAVE) {  // d = 1024: lane l holds elements 16l..16l+15 (two 16-B loads)
      const int4* p = reinterpret_cast<const int4*>(x + 16 * l);
      const int4 a = p[0], b = p[1];
      const uint32_t wv[8] = {(uint32_t)a.x, (uint32_t)a.y, (uint32_t)a.z, (uint32_t)a.w,
                              (uint32_t)b.x, (uint32_t)b.y, (uint32_t)b.z, (uint32_t)b.w};
      int e[16];
      int32_t ls = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        e[k] = (int)(int16_t)(wv[k >> 1] >> (16 * (k & 1)));
        ls += e[k];
      }
      const double mean = (double)wave_sum_i64((int64_t)ls) / (double)dim;  // exact sum, one rounding
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) bits |= ((double)e[k] > mean ? 1u : 0u) << ((k < 8 ? 7 - k : 23 - k));
      *reinterpret_cast<uint16_t*>(crow + 2 * l) = (uint16_t)bits;  // bytes 2l (elements 0..7), 2l+1
      return;
    }
    int64_t s = 0;
    for (int i = l; i < dim; i += WAVE) s += x[i];
    s = wave_sum_i64(s);
    const double mean = (double)s / (double)dim;
    for (int gi = l; gi < ngroups; gi += WAVE) {
      uint32_t byte = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) byte |= ((double)x[8 * gi + k] > mean ? 1u : 0u) << (7 - k);
      crow[gi] = (uint8_t)byte;
    }
    return;
  } else {
    const float* x = reinterpret_cast<const float*>(xin) + v * dim;
    for (int i = 4 * l; i < dim; i += 4 * WAVE) *reinterpret_cast<float4*>(xs + i) = *reinterpret_cast<const float4*>(x + i);
    wave_lds_sync();
    float mean = 0.f;
    if constexpr (MODE != VRQ_ENC_COHERE) {
      const float s = pairwise_sum_f32(xs, P, leafsum);
      mean = (float)((double)s / (double)dim);  // np.float32(sum) / np.intp(n) -> float32
    }
    float mn = __builtin_inff(), mx = -__builtin_inff();
    if constexpr (MODE == VRQ_ENC_INT4_GLOBAL || MODE == VRQ_ENC_INT8_LOCAL || MODE == VRQ_ENC_INT4_LOCAL) {
      for (int i = l; i < dim; i += WAVE) {
        mn = fminf(mn, xs[i]);
        mx = fmaxf(mx, xs[i]);
      }
#pragma unroll
      for (int m = 1; m < WAVE; m <<= 1) {
        mn = fminf(mn, __shfl_xor(mn, m, WAVE));
        mx = fmaxf(mx, __shfl_xor(mx, m, WAVE));
      }
      if constexpr (MODE != VRQ_ENC_INT4_GLOBAL) {
        if (l == 0) {
          minmax[2 * v] = (double)mn;
          minmax[2 * v + 1] = (double)mx;
        }
      }
    }
    const float am = fmaxf(fabsf(mn), fabsf(mx));
    const bool flat = (mx == mn);
    float scale = 0.f, lim = 0.f;
    if constexpr (MODE == VRQ_ENC_INT8_GLOBAL || MODE == VRQ_ENC_COHERE) {
      lim = (float)limit;
      scale = (float)(127.0 / limit);
    } else if constexpr (MODE == VRQ_ENC_INT16_GLOBAL) {
      lim = (float)limit;
      scale = (float)(32767.0 / limit);
    } else if constexpr (MODE == VRQ_ENC_INT8_LOCAL) {
      scale = flat ? 0.f : (float)(127.0 / (double)am);
    } else {
      scale = flat ? 0.f : (float)(7.0 / (double)am);
    }
    for (int gi = l; gi < ngroups; gi += WAVE) {
      float e[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = xs[8 * gi + k];
      uint32_t byte = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const bool bit = (MODE == VRQ_ENC_COHERE) ? (e[k] > 0.f) : (e[k] > mean);
        byte |= (bit ? 1u : 0u) << (7 - k);
      }
      crow[gi] = (uint8_t)byte;
      if constexpr (MODE == VRQ_ENC_INT8_GLOBAL || MODE == VRQ_ENC_COHERE) {
        uint32_t w[2] = {0, 0};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float y = clampf(rintf(clampf(e[k], -lim, lim) * scale), -127.f, 127.f);
          w[k >> 2] |= ((uint32_t)(uint8_t)(int8_t)(int)y) << (8 * (k & 3));
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<int8_t*>(qout) + v * dim + 8 * gi) = make_uint2(w[0], w[1]);
      } else if constexpr (MODE == VRQ_ENC_INT16_GLOBAL) {
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float y = clampf(rintf(clampf(e[k], -lim, lim) * scale), -32767.f, 32767.f);
          w[k >> 1] |= ((uint32_t)(uint16_t)(int16_t)(int)y) << (16 * (k & 1));
        }
        *reinterpret_cast<uint4*>(reinterpret_cast<int16_t*>(qout) + v * dim + 8 * gi) =
            make_uint4(w[0], w[1], w[2], w[3]);
      } else if constexpr (MODE == VRQ_ENC_INT8_LOCAL) {
        uint32_t w[2] = {0, 0};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int y = flat ? 0 : (int)(e[k] * scale);  // astype(int8): truncation toward zero
          w[k >> 2] |= ((uint32_t)(uint8_t)(int8_t)y) << (8 * (k & 3));
        }
        *reinterpret_cast<uint2*>(reinterpret_cast<int8_t*>(qout) + v * dim + 8 * gi) = make_uint2(w[0], w[1]);
      } else {  // int4 (global: limit ignored; local): nibble pairs, high = even index
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < 8; k += 2) {
          uint32_t byte4 = 0;
          if (!flat) {
            const int a = (int)clampf(rintf(e[k] * scale), -8.f, 7.f) + 8;
            const int b = (int)clampf(rintf(e[k + 1] * scale), -8.f, 7.f) + 8;
            byte4 = (uint32_t)(((a & 0x0f) << 4) | (b & 0x0f));
          }
          w |= byte4 << (8 * (k >> 1));
        }
        *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(qout) + v * (dim / 2) + 4 * gi) = w;
      }
    }
  }
}

// d = 1024 float modes (every BASELINE shape): persistent waves, each looping over vectors
// v = gw, gw + nw, ...; the next vector's 4 KiB is loaded into registers while the current one is
// encoded.  Lane l holds elements 256k + 4l + c (k, c < 4: four coalesced 1 KiB loads).
//  * mean: the 4 KiB go to the wave's LDS slice once; lane 8g + j accumulates leaf g's column j
//    (16 sequential adds, NumPy's order), then a 6-step butterfly (xor 1, 2, 4: the leaf's
//    ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)); xor 8, 16, 32: the balanced tree over the 8 leaves) leaves
//    the exact pairwise sum in every lane (each step adds the same two values in every lane pair);
//  * min / max (local modes) and the quantised outputs come from the registers: q bytes / int16 /
//    nibbles of elements 256k + 4l + c are stored per k as one coalesced 256 / 512 / 128 B row;
//  * the code bytes from the LDS slice: lane l packs elements 16l..16l+15 (four conflict-free
//    ds_read_b128) into bytes 2l, 2l+1 (one 128 B store per wave).
constexpr int ENC_WPB = 4;                       // waves per workgroup (each on its own LDS slice)
constexpr int ENC_SLICE = 1024 + 64;             // floats per wave slice (+ padding)

// One butterfly step without the LDS crossbar (a __shfl_xor is a ds_bpermute round trip, ~100+
// cycles on the wave's critical path): lane l combines its value with lane l ^ M's.  M = 1, 2: quad
// DPP; M = 4, 8: the half-row / row mirror DPP, which pair lane l with a lane of the group l ^ M
// once every group of M lanes holds a single value (true after the steps below M); M = 16, 32:
// v_permlane16/32_swap, which hand every lane both values of the pair.  OP is commutative, so each
// lane computes the same value as OP(own, partner) of the __shfl_xor butterfly (bit-exact).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
template <int M, class OP>
__device__ __forceinline__ float bfly(float x, OP op) {
  if constexpr (M == 1) {
    return op(x, dpp_mov<0xB1>(x));  // quad_perm [1,0,3,2]
  } else if constexpr (M == 2) {
    return op(x, dpp_mov<0x4E>(x));  // quad_perm [2,3,0,1]
  } else if constexpr (M == 4) {
    return op(x, dpp_mov<0x141>(x));  // row_half_mirror
  } else if constexpr (M == 8) {
    return op(x, dpp_mov<0x140>(x));  // row_mirror
  } else if constexpr (M == 16) {
    const auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return op(__uint_as_float(p[0]), __uint_as_float(p[1]));
  } else {
    static_assert(M == 32, "butterfly step");
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
    return op(__uint_as_float(p[0]), __uint_as_float(p[1]));
  }
}
template <class OP>
__device__ __forceinline__ float wave_allreduce(float x, OP op) {
  x = bfly<1>(x, op);
  x = bfly<2>(x, op);
  x = bfly<4>(x, op);
  x = bfly<8>(x, op);
  x = bfly<16>(x, op);
  return bfly<32>(x, op);
}

// Input rows by non-temporal loads (each f32 row is read once) for the modes where that measured
// faster: int8g 0.66 -> 0.71, int16g 0.70 -> 0.71, Cohere 0.71 -> 0.72 of HBM; int4g and the local
// modes measured 0.01-0.02 slower with it (tools/enc_probe.py, profiles/r3_encode_nt_variants.jsonl).
template <int MODE>
constexpr bool enc_nt() {
  return MODE == VRQ_ENC_INT8_GLOBAL || MODE == VRQ_ENC_INT16_GLOBAL || MODE == VRQ_ENC_COHERE;
}
template <int MODE>
__device__ __forceinline__ void enc1024_load(float4 (&x)[4], const float* __restrict__ row, int l) {
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if constexpr (enc_nt<MODE>()) {
      typedef float f4v __attribute__((ext_vector_type(4)));
      const f4v v = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(row + 256 * k + 4 * l));
      x[k] = make_float4(v.x, v.y, v.z, v.w);
    } else {
      x[k] = *reinterpret_cast<const float4*>(row + 256 * k + 4 * l);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(ENC_WPB * 64) void encode1024_kernel(const float* __restrict__ xin, int64_t n,
                                                                  double limit, uint8_t* __restrict__ codes,
                                                                  void* __restrict__ qout, double* __restrict__ minmax) {
  __shared__ __attribute__((aligned(16))) float smem[ENC_WPB * ENC_SLICE];
  const int w = threadIdx.x >> 6, l = lane_id(), g = l >> 3, j = l & 7;
  float* xs = smem + w * ENC_SLICE;
  const int64_t v = (int64_t)blockIdx.x * ENC_WPB + w;  // one vector per wave
  if (v >= n) return;
  float4 xc[4];
  enc1024_load<MODE>(xc, xin + v * 1024, l);
  float lim = 0.f, gscale = 0.f;
  if constexpr (MODE == VRQ_ENC_INT8_GLOBAL || MODE == VRQ_ENC_COHERE) {
    lim = (float)limit;
    gscale = (float)(127.0 / limit);
  } else if constexpr (MODE == VRQ_ENC_INT16_GLOBAL) {
    lim = (float)limit;
    gscale = (float)(32767.0 / limit);
  }
  {
    float e[16];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[4 * k] = xc[k].x;
      e[4 * k + 1] = xc[k].y;
      e[4 * k + 2] = xc[k].z;
      e[4 * k + 3] = xc[k].w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) *reinterpret_cast<float4*>(xs + 256 * k + 4 * l) = xc[k];
    wave_lds_sync();
    float mean = 0.f;
    if constexpr (MODE != VRQ_ENC_COHERE) {
      const float* leaf = xs + 128 * g + j;
      float r = leaf[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) r += leaf[8 * i];
      r = wave_allreduce(r, [](float a, float b) { return a + b; });
      mean = (float)((double)r / 1024.0);  // np.float32(sum) / np.intp(n) -> float32
    }
    // code bytes 2l, 2l+1 = elements 16l..16l+15 (MSB first)
    {
      const float4* p = reinterpret_cast<const float4*>(xs + 16 * l);
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float4 c = p[k];
        const float cv[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int idx = 4 * k + q;  // element 16l + idx -> byte idx / 8, bit 7 - idx % 8
          const bool bit = (MODE == VRQ_ENC_COHERE) ? (cv[q] > 0.f) : (cv[q] > mean);
          bits |= (bit ? 1u : 0u) << ((idx < 8) ? 7 - idx : 23 - idx);
        }
      }
      *reinterpret_cast<uint16_t*>(codes + v * 128 + 2 * l) = (uint16_t)bits;
    }
    float scale = gscale;
    bool flat = false;
    if constexpr (MODE == VRQ_ENC_INT4_GLOBAL || MODE == VRQ_ENC_INT8_LOCAL || MODE == VRQ_ENC_INT4_LOCAL) {
      // min / max as v_med3 against -+inf (no NaN canonicalisation per element).  Inputs must be
      // finite (include/vrq.h): a NaN element makes v_med3 return the min3 of its operands, so
      // mn = -inf and the local code is all zero; the generic kernel's fminf/fmaxf ignore NaNs.  The
      // reference has no defined NaN result to match (NumPy min/max/mean propagate NaN into the cast).
      float mn = e[0], mx = e[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) {
        mn = __builtin_amdgcn_fmed3f(mn, e[i], -__builtin_inff());
        mx = __builtin_amdgcn_fmed3f(mx, e[i], __builtin_inff());
      }
      mn = wave_allreduce(mn, [](float a, float b) { return __builtin_amdgcn_fmed3f(a, b, -__builtin_inff()); });
      mx = wave_allreduce(mx, [](float a, float b) { return __builtin_amdgcn_fmed3f(a, b, __builtin_inff()); });
      if constexpr (MODE != VRQ_ENC_INT4_GLOBAL) {
        if (l == 0) {
          minmax[2 * v] = (double)mn;
          minmax[2 * v + 1] = (double)mx;
        }
      }
      const float am = fmaxf(fabsf(mn), fabsf(mx));
      flat = (mx == mn);
      scale = flat ? 0.f : (float)((MODE == VRQ_ENC_INT8_LOCAL ? 127.0 : 7.0) / (double)am);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float* ek = e + 4 * k;
      const int64_t o = v * 1024 + 256 * k + 4 * l;  // element index of ek[0]
      // (clamps as v_med3 -- no NaN canonicalisation; round half to even = v_rndne; integer-valued
      // results are packed by v_cvt_pk_u8_f32 after a +128 / +8 bias, which is exact for them)
      if constexpr (MODE == VRQ_ENC_INT8_GLOBAL || MODE == VRQ_ENC_COHERE) {
        uint32_t wd = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float y = __builtin_amdgcn_fmed3f(
              __builtin_rintf(__builtin_amdgcn_fmed3f(ek[c], -lim, lim) * scale), -127.f, 127.f);
          wd = __builtin_amdgcn_cvt_pk_u8_f32(y + 128.f, c, wd);
        }
        *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(qout) + o) = wd ^ 0x80808080u;  // biased -> int8
      } else if constexpr (MODE == VRQ_ENC_INT16_GLOBAL) {
        int y[4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
          y[c] = (int)__builtin_amdgcn_fmed3f(__builtin_rintf(__builtin_amdgcn_fmed3f(ek[c], -lim, lim) * scale),
                                              -32767.f, 32767.f);
        typedef short s2v __attribute__((ext_vector_type(2)));
        const s2v lo = __builtin_amdgcn_cvt_pk_i16(y[0], y[1]), hi = __builtin_amdgcn_cvt_pk_i16(y[2], y[3]);
        *reinterpret_cast<uint2*>(reinterpret_cast<int16_t*>(qout) + o) =
            make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
      } else if constexpr (MODE == VRQ_ENC_INT8_LOCAL) {
        uint32_t wd = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int y = flat ? 0 : (int)(ek[c] * scale);  // astype(int8): truncation toward zero
          wd |= ((uint32_t)(uint8_t)(int8_t)y) << (8 * c);
        }
        *reinterpret_cast<uint32_t*>(reinterpret_cast<int8_t*>(qout) + o) = wd;
      } else {  // int4: nibble pairs, high = even index; bytes (o / 2), (o / 2) + 1
        uint32_t bw = 0;  // biased values 0..15 of elements c = 0..3 in bytes 0..3
#pragma unroll
        for (int c = 0; c < 4; ++c)
          bw = __builtin_amdgcn_cvt_pk_u8_f32(__builtin_amdgcn_fmed3f(__builtin_rintf(ek[c] * scale), -8.f, 7.f) + 8.f,
                                              c, bw);
        // bytes (a0, b0, a1, b1) -> (a0 << 4 | b0, a1 << 4 | b1)
        const uint32_t t = ((bw & 0x00ff00ffu) << 4) | ((bw >> 8) & 0x00ff00ffu);
        const uint32_t hw = flat ? 0u : ((t & 0xffu) | ((t >> 8) & 0xff00u));
        *reinterpret_cast<uint16_t*>(reinterpret_cast<int8_t*>(qout) + o / 2) = (uint16_t)hw;
      }
    }
  }
}

// K7: ||x8 row||_2 in float64 from the exact integer sum of squares.
__global__ __launch_bounds__(256) void int8_norms_kernel(const int8_t* __restrict__ x8, int64_t n, int dim,
                                                         double* __restrict__ out) {
  // grid-stride over rows, one wave per row: the grid stays far below the 2^32 work-item limit of a
  // dispatch at 100M rows
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int l = lane_id();
  for (int64_t v = ((int64_t)blockIdx.x * 256 + threadIdx.x) / WAVE; v < n; v += nw) {
    const int8_t* r = x8 + v * dim;
    int64_t s = 0;
    if ((dim & 15) == 0) {
      for (int i = 16 * l; i < dim; i += 16 * WAVE) {
        const int4 raw = *reinterpret_cast<const int4*>(r + i);
        const int32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int32_t e = (int8_t)((w[k >> 2] >> (8 * (k & 3))) & 0xff);
          s += e * e;
        }
      }
    } else {
      for (int i = l; i < dim; i += WAVE) s += (int32_t)r[i] * (int32_t)r[i];
    }
    s = wave_sum_i64(s);
    if (l == 0) out[v] = sqrt((double)s);
  }
}

}  // namespace vrq

using namespace vrq;

extern "C" {

int vrq_abi_version(void) { return VRQ_ABI_VERSION; }

const char* vrq_strerror(int code) {
  switch (code) {
    case VRQ_OK: return "ok";
    case VRQ_EINVAL: return "invalid argument";
    case VRQ_EHIP: return "HIP runtime error";
    case VRQ_EUNSUPPORTED: return "unsupported shape";
    case VRQ_EWORKSPACE: return "workspace too small";
    default: return "unknown vrq error";
  }
}

int vrq_encode(int32_t mode, const void* x, int64_t n, int32_t dim, double limit, uint8_t* codes, void* q,
               double* minmax, void* stream) {
  VRQ_CHECK_ARG(n >= 0 && dim > 0 && (dim % 8) == 0);
  if (dim > MAX_DIM || (dim % 4) != 0) return VRQ_EUNSUPPORTED;
  VRQ_CHECK_ARG(mode >= VRQ_ENC_INT8_GLOBAL && mode <= VRQ_ENC_COHERE);
  const bool global_mode = mode == VRQ_ENC_INT8_GLOBAL || mode == VRQ_ENC_INT16_GLOBAL || mode == VRQ_ENC_COHERE;
  if (global_mode) VRQ_CHECK_ARG(limit > 0.0);
  if (n == 0) return VRQ_OK;
  VRQ_CHECK_ARG(x && codes);
  if (mode != VRQ_ENC_BIN_INT16) VRQ_CHECK_ARG(q);
  if (mode == VRQ_ENC_INT8_LOCAL || mode == VRQ_ENC_INT4_LOCAL) VRQ_CHECK_ARG(minmax);
  PwPlan P{};
  pw_build(0, dim, &P);
  pw_classify(&P);
  if (P.nleaves > MAX_LEAVES) return VRQ_EUNSUPPORTED;
  // EPB vectors per workgroup while their LDS slices stay within 64 KiB (dim <= 3840), else one
  const int epb = sizeof(float) * EPB * (dim + 2 * MAX_LEAVES) <= 65536 ? EPB : 1;
  const size_t lds = sizeof(float) * epb * (dim + 2 * MAX_LEAVES);
  hipStream_t s = (hipStream_t)stream;
  // one wave per vector (EPB per workgroup); launches of at most 2^24 vectors keep a dispatch below
  // 2^32 work-items
  const int64_t xrow = (int64_t)dim * (mode == VRQ_ENC_BIN_INT16 ? 2 : 4);
  const int64_t qrow = mode == VRQ_ENC_INT16_GLOBAL                              ? 2 * (int64_t)dim
                       : (mode == VRQ_ENC_INT4_GLOBAL || mode == VRQ_ENC_INT4_LOCAL) ? (int64_t)(dim + 1) / 2
                                                                                    : (int64_t)dim;
  if (dim == 1024 && mode != VRQ_ENC_BIN_INT16) {
    // one vector per wave (the measured best: 0.63-0.71 of HBM vs 0.58-0.61 for 4-6 persistent
    // workgroups per CU, tools/enc_probe.py), launches of at most 2^22 workgroups (2^24 vectors, a
    // dispatch below 2^32 work-items)
    const int64_t wgs = (n + ENC_WPB - 1) / ENC_WPB;
    constexpr int64_t kMaxWgs = int64_t(1) << 22;
    const int64_t lw = wgs > kMaxWgs ? kMaxWgs : wgs;  // workgroups' vectors per launch
    for (int64_t w0 = 0; w0 < wgs; w0 += lw) {
    const int64_t v0 = w0 * ENC_WPB, nv = n - v0 < lw * ENC_WPB ? n - v0 : lw * ENC_WPB;
    const int64_t g = (nv + ENC_WPB - 1) / ENC_WPB;
    const dim3 grid((unsigned)g), block(ENC_WPB * 64);
    const float* xf = (const float*)x + v0 * 1024;
    uint8_t* cv = codes + v0 * 128;
    void* qv = (uint8_t*)q + v0 * qrow;
    double* mv = minmax ? minmax + 2 * v0 : nullptr;
    switch (mode) {
      case VRQ_ENC_INT8_GLOBAL:
        hipLaunchKernelGGL(encode1024_kernel<VRQ_ENC_INT8_GLOBAL>, grid, block, 0, s, xf, nv, limit, cv, qv, mv);
        break;
      case VRQ_ENC_INT16_GLOBAL:
        hipLaunchKernelGGL(encode1024_kernel<VRQ_ENC_INT16_GLOBAL>, grid, block, 0, s, xf, nv, limit, cv, qv, mv);
        break;
      case VRQ_ENC_INT4_GLOBAL:
        hipLaunchKernelGGL(encode1024_kernel<VRQ_ENC_INT4_GLOBAL>, grid, block, 0, s, xf, nv, limit, cv, qv, mv);
        break;
      case VRQ_ENC_INT8_LOCAL:
        hipLaunchKernelGGL(encode1024_kernel<VRQ_ENC_INT8_LOCAL>, grid, block, 0, s, xf, nv, limit, cv, qv, mv);
        break;
      case VRQ_ENC_INT4_LOCAL:
        hipLaunchKernelGGL(encode1024_kernel<VRQ_ENC_INT4_LOCAL>, grid, block, 0, s, xf, nv, limit, cv, qv, mv);
        break;
      default:
        hipLaunchKernelGGL(encode1024_kernel<VRQ_ENC_COHERE>, grid, block, 0, s, xf, nv, limit, cv, qv, mv);
        break;
    }
    VRQ_LAUNCH_CHECK();
    }
    return VRQ_OK;
  }
  constexpr int64_t kMaxLaunch = 1 << 24;
  for (int64_t v0 = 0; v0 < n; v0 += kMaxLaunch) {
    const int64_t nv = n - v0 < kMaxLaunch ? n - v0 : kMaxLaunch;
    const void* xv = (const uint8_t*)x + v0 * xrow;
    uint8_t* cv = codes + v0 * (dim / 8);
    void* qv = q ? (void*)((uint8_t*)q + v0 * qrow) : nullptr;
    double* mv = minmax ? minmax + 2 * v0 : nullptr;
    const dim3 grid((unsigned)((nv + epb - 1) / epb)), block(epb * 64);
    switch (mode) {
      case VRQ_ENC_INT8_GLOBAL:
        hipLaunchKernelGGL(encode_kernel<VRQ_ENC_INT8_GLOBAL>, grid, block, lds, s, xv, nv, dim, limit, cv, qv, mv, P, epb);
        break;
      case VRQ_ENC_INT16_GLOBAL:
        hipLaunchKernelGGL(encode_kernel<VRQ_ENC_INT16_GLOBAL>, grid, block, lds, s, xv, nv, dim, limit, cv, qv, mv, P, epb);
        break;
      case VRQ_ENC_INT4_GLOBAL:
        hipLaunchKernelGGL(encode_kernel<VRQ_ENC_INT4_GLOBAL>, grid, block, lds, s, xv, nv, dim, limit, cv, qv, mv, P, epb);
        break;
      case VRQ_ENC_INT8_LOCAL:
        hipLaunchKernelGGL(encode_kernel<VRQ_ENC_INT8_LOCAL>, grid, block, lds, s, xv, nv, dim, limit, cv, qv, mv, P, epb);
        break;
      case VRQ_ENC_INT4_LOCAL:
        hipLaunchKernelGGL(encode_kernel<VRQ_ENC_INT4_LOCAL>, grid, block, lds, s, xv, nv, dim, limit, cv, qv, mv, P, epb);
        break;
      case VRQ_ENC_BIN_INT16:
        hipLaunchKernelGGL(encode_kernel<VRQ_ENC_BIN_INT16>, grid, block, lds, s, xv, nv, dim, limit, cv, qv, mv, P, epb);
        break;
      default:
        hipLaunchKernelGGL(encode_kernel<VRQ_ENC_COHERE>, grid, block, lds, s, xv, nv, dim, limit, cv, qv, mv, P, epb);
        break;
    }
    VRQ_LAUNCH_CHECK();
  }
  return VRQ_OK;
}

int vrq_int8_row_norms(const int8_t* x8, int64_t n, int32_t dim, double* out, void* stream) {
  VRQ_CHECK_ARG(n >= 0 && dim > 0);
  if (n == 0) return VRQ_OK;
  VRQ_CHECK_ARG(x8 && out);
  int64_t blocks = (n * WAVE + 255) / 256;
  if (blocks > (1 << 20)) blocks = 1 << 20;  // 4M waves, grid-stride beyond
  hipLaunchKernelGGL(int8_norms_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, x8, n, dim, out);
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

}  // extern "C"
