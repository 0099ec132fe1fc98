// select_rescore.hip -- K2: exact merge of the per-chunk Phase-I lists + fused
// Phase II / Phase III rescoring and the reference's stable sorts, one
// 256-thread workgroup per query.  Also the shard merge used after the RCCL
// all-gather (vrq_merge_shards) and the stand-alone rescoring entry points.
//
// Reference semantics (CohereEnhancedVectorDB.py):
//   :267-275  K = binary_k Phase-I hits in FAISS (dist asc, row asc) order
//   :283-293  s2 = float(qf . (2*unpackbits(code)-1))   float32.int32 -> float64
//   :296-297  stable sort by s2 desc, keep K3 = k*int8_oversample
//   :302-318  s3 = float(qf . int8) / np.linalg.norm(int8); -inf if norm == 0
//   :321-322  stable sort by s3 desc, first k
// Numerics: Phase II is accumulated in float64 -- every product is +-q_i
// (exact) and the partial sums of float32 embedding values fit in 53 bits, so
// the sum is exact and equals NumPy's ddot bit for bit.  Phase III: the f32
// x int8 products are exact in float64 and so is their sum; rounding it once
// to float32 gives the correctly rounded float32 dot (NumPy's sdot rounds per
// BLAS summation order, <= a few ulp away: the 1e-5 tolerance of the north
// star).  The norm is sqrt of an exact integer sum (correctly rounded, equal
// to np.linalg.norm) and the division is IEEE double, as in the reference.
#include "exact_scores.h"
#include "vrq_internal.h"
#include "vrq_scan.h"

namespace vrq {

constexpr int SEL_THREADS = 256;
constexpr int KMAX = 1024;          // max K (binary_k) handled per query
constexpr int MAX_LISTS = 4096;     // max chunk lists merged per query
constexpr int NBINS = 1025 + 3;     // dist in [0, 1024] for 1024-bit codes
constexpr uint64_t ROW_MASK = (1ull << KEY_ROW_BITS) - 1;

// Per-query LDS state, sized for at most KM candidates (binary_k) and ML lists.  The general
// instance (KMAX, MAX_LISTS) takes ~89 KiB, one workgroup per CU; the common shape (K <= 128,
// <= 64 lists) runs the small instance (~11 KiB) so 8 workgroups share a CU.
template <int KM, int ML>
struct SelShared {
  static constexpr int kKM = KM, kML = ML;
  uint32_t hist[NBINS];
  int32_t ltcnt[ML];
  int32_t eqend[ML];
  uint64_t sel[KM];         // Phase-I keys (dist << 40 | row), FAISS order after select
  int32_t pay[KM];          // payload index (list * K + pos) of each selected key
  uint64_t skey[KM];        // sort keys (descending score image)
  int32_t sidx[KM];         // sort payload (Phase-I rank)
  double s2[KM];
  double s3[KM];
  int32_t ord2[KM];         // Phase-I ranks in Phase-II order (first K3)
  double s3o[KM];           // Phase-III scores in Phase-II order
  int32_t scan[SEL_THREADS / WAVE + 1];
  int32_t misc[8];
};
constexpr int KSMALL = 128, LSMALL = 64;
typedef SelShared<KMAX, MAX_LISTS> SelBig;
typedef SelShared<KSMALL, LSMALL> SelSmall;

// Block-wide exclusive scan of one int per thread; returns exclusive prefix, total in *tot.
__device__ inline int block_excl_scan(int v, int* tot, int32_t* scratch) {
  const int l = lane_id(), w = threadIdx.x / WAVE;
  int x = v;
#pragma unroll
  for (int o = 1; o < WAVE; o <<= 1) {
    const int y = __shfl_up(x, o, WAVE);
    if (l >= o) x += y;
  }
  __syncthreads();
  if (l == WAVE - 1) scratch[w] = x;
  __syncthreads();
  int base = 0, all = 0;
  for (int i = 0; i < SEL_THREADS / WAVE; ++i) {
    const int s = scratch[i];
    if (i < w) base += s;
    all += s;
  }
  __syncthreads();
  *tot = all;
  return base + x - v;
}

// Exact top-Kp (Kp = min(K, #valid)) of the union of nl sorted lists of K keys each,
// whose row ranges are disjoint and increasing with the list index.  Result: sh.sel[0..Kp)
// ascending by key (= FAISS (dist, row) order) with sh.pay = list*K + pos.  Returns Kp.
template <class KeyAt, class SH>
__device__ int select_topk(const KeyAt& L, int nl, int K, SH& sh) {
  const int tid = threadIdx.x;
  const int total = nl * K;
  for (int i = tid; i < NBINS; i += SEL_THREADS) sh.hist[i] = 0;
  for (int i = tid; i < nl; i += SEL_THREADS) {
    sh.ltcnt[i] = 0;
    sh.eqend[i] = 0;
  }
  __syncthreads();
  for (int i = tid; i < total; i += SEL_THREADS) {
    const uint64_t key = L[i];
    const uint32_t d = (uint32_t)(key >> KEY_ROW_BITS);
    if (key != KEY_NONE && d < (uint32_t)NBINS) atomicAdd(&sh.hist[d], 1u);
  }
  __syncthreads();
  // threshold T: smallest d with cum(d) >= Kp
  constexpr int BPT = (NBINS + SEL_THREADS - 1) / SEL_THREADS;
  int local = 0;
  for (int b = 0; b < BPT; ++b) {
    const int i = tid * BPT + b;
    if (i < NBINS) local += (int)sh.hist[i];
  }
  int valid = 0;
  int pre = block_excl_scan(local, &valid, sh.scan);
  const int Kp = K < valid ? K : valid;
  if (tid == 0) {
    sh.misc[0] = 0x7fffffff;
    sh.misc[1] = 0;
  }
  __syncthreads();
  if (Kp == 0) return 0;
  {
    int cum = pre;
    for (int b = 0; b < BPT; ++b) {
      const int i = tid * BPT + b;
      if (i >= NBINS) break;
      const int h = (int)sh.hist[i];
      if (cum < Kp && cum + h >= Kp) {
        sh.misc[0] = i;    // T
        sh.misc[1] = cum;  // c_lt = #entries with dist < T
      }
      cum += h;
    }
  }
  __syncthreads();
  const uint32_t T = (uint32_t)sh.misc[0];
  const int c_lt = sh.misc[1];
  const int R = Kp - c_lt;  // entries with dist == T to take, in row order
  // per-list lt / eq run ends (each list is sorted by (dist,row))
  for (int i = tid; i < total; i += SEL_THREADS) {
    const int c = i / K, p = i - c * K;
    const uint32_t d = (uint32_t)(L[i] >> KEY_ROW_BITS);
    const uint32_t dn = (p + 1 < K) ? (uint32_t)(L[i + 1] >> KEY_ROW_BITS) : 0xffffffffu;
    if (d < T && dn >= T) sh.ltcnt[c] = p + 1;
    if (d == T && dn != T) sh.eqend[c] = p + 1;
  }
  __syncthreads();
  // exclusive scans over lists of lt counts and eq counts (LPT lists per thread)
  const int LPT = (nl + SEL_THREADS - 1) / SEL_THREADS;
  int sl = 0, se = 0;
  for (int b = 0; b < LPT; ++b) {
    const int c = tid * LPT + b;
    if (c < nl) {
      const int lt = sh.ltcnt[c];
      const int eq = sh.eqend[c] > lt ? sh.eqend[c] - lt : 0;
      sl += lt;
      se += eq;
    }
  }
  int tl, te;
  int pl = block_excl_scan(sl, &tl, sh.scan);
  int pe = block_excl_scan(se, &te, sh.scan);
  // convert ltcnt/eqend into (lt prefix, eq prefix - lt) in place, per thread range
  for (int b = 0; b < LPT; ++b) {
    const int c = tid * LPT + b;
    if (c < nl) {
      const int lt = sh.ltcnt[c];
      const int eq = sh.eqend[c] > lt ? sh.eqend[c] - lt : 0;
      sh.ltcnt[c] = pl;       // output base of this list's dist<T run
      sh.eqend[c] = pe - lt;  // rank of entry p (dist==T) = eqend[c] + p
      pl += lt;
      pe += eq;
    }
  }
  __syncthreads();
  for (int i = tid; i < total; i += SEL_THREADS) {
    const uint64_t key = L[i];
    const uint32_t d = (uint32_t)(key >> KEY_ROW_BITS);
    if (d > T) continue;
    const int c = i / K, p = i - c * K;
    if (d < T) {
      const int o = sh.ltcnt[c] + p;
      sh.sel[o] = key;
      sh.pay[o] = i;
    } else {
      const int r = sh.eqend[c] + p;
      if (r < R) {
        sh.sel[c_lt + r] = key;
        sh.pay[c_lt + r] = i;
      }
    }
  }
  __syncthreads();
  // sort the dist<T group (the dist==T group is already in row order)
  if (c_lt > 1) {
    const int np2 = next_pow2(c_lt);
    for (int i = c_lt + tid; i < np2; i += SEL_THREADS) {
      sh.skey[i] = KEY_NONE;
    }
    for (int i = tid; i < c_lt; i += SEL_THREADS) {
      sh.skey[i] = sh.sel[i];
      sh.sidx[i] = sh.pay[i];
    }
    block_bitonic_sort_kv(sh.skey, sh.sidx, np2);
    for (int i = tid; i < c_lt; i += SEL_THREADS) {
      sh.sel[i] = sh.skey[i];
      sh.pay[i] = sh.sidx[i];
    }
  }
  __syncthreads();
  return Kp;
}

// Stable descending sort of scores sc[0..m) keeping the original positions:
// (desc image of score, position) lexicographic -- Python's list.sort(reverse=True)
// on a key is stable, so equal scores keep their previous order (:296, :321).
template <class SH>
__device__ void stable_desc_order(const double* sc, int m, SH& sh) {
  if (m <= SEL_THREADS) {
    // one element per thread: its rank = #{j : (key_j, j) < (key_i, i)} over the m keys (broadcast LDS
    // reads), then one scatter -- 3 barriers instead of a bitonic network's log^2 rounds of them
    const int i = threadIdx.x;
    const uint64_t ki = i < m ? desc_key_f64(sc[i]) : KEY_NONE;
    if (i < m) sh.skey[i] = ki;
    __syncthreads();
    int rank = 0;
    if (i < m)
      for (int j = 0; j < m; ++j) {
        const uint64_t kj = sh.skey[j];
        rank += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
      }
    __syncthreads();
    if (i < m) {
      sh.skey[rank] = ki;
      sh.sidx[rank] = i;
    }
    __syncthreads();
    return;
  }
  const int np2 = next_pow2(m > 1 ? m : 1);
  for (int i = threadIdx.x; i < np2; i += SEL_THREADS) {
    sh.skey[i] = i < m ? desc_key_f64(sc[i]) : KEY_NONE;
    sh.sidx[i] = i < m ? i : 0x7fffffff;
  }
  // bitonic on (skey, sidx) lexicographic
  for (int size = 2; size <= np2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < (np2 >> 1); i += SEL_THREADS) {
        const int lo = ((i / stride) * stride * 2) + (i % stride);
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t ka = sh.skey[lo], kb = sh.skey[hi];
        const int ia = sh.sidx[lo], ib = sh.sidx[hi];
        const bool gt = (ka > kb) || (ka == kb && ia > ib);
        if (gt == up) {
          sh.skey[lo] = kb;
          sh.skey[hi] = ka;
          sh.sidx[lo] = ib;
          sh.sidx[hi] = ia;
        }
      }
    }
  }
  __syncthreads();
}

// Finish one query from Phase-I candidates sh.sel[0..Kp) with s2 (and s3 where needed)
// already in sh.s2/sh.s3 by Phase-I rank: stable sort by s2, cut K3, stable sort by
// s3, cut k, write outputs.  have_s3: s3 valid for all Kp (shard merge); otherwise
// it is computed here for the K3 survivors.
struct FinishArgs {
  const float* q;
  const int8_t* x8;
  const double* norms;
  const int64_t* remap;  // rescore row of each Phase-I row (IDMap2 rev_map[id_map[r]]), or null
  int64_t row_offset;  // added to local rows for output
  int k, K3;
  int32_t* out_count;
  int64_t* out_rows;
  int32_t* out_dist;
  double* out_s2;
  double* out_s3;
  int32_t* out_src;  // shard merge only: payload index (shard * K + pos) of each output, or null
  int kout;
};

template <class SH>
__device__ void finish_query(int Kp, bool have_s3, const FinishArgs& a, int qi, SH& sh) {
  const int tid = threadIdx.x, w = tid / WAVE, l = lane_id();
  stable_desc_order(sh.s2, Kp, sh);  // sh.sidx[0..Kp) = Phase-I ranks in Phase-II order
  const int K3p = a.K3 < Kp ? a.K3 : Kp;
  // stash the Phase-II order (sidx is reused by the next sort)
  int32_t* ord2 = sh.ord2;
  for (int i = tid; i < K3p; i += SEL_THREADS) ord2[i] = sh.sidx[i];
  __syncthreads();
  if (!have_s3) {
    float qv[DPL];
    load_q(qv, a.q);
    // CB3 survivors per wave in flight: every row's load issued before the first score.  The loads are
    // unconditional (indices past K3p re-read the last survivor): a load under a divergent branch gets
    // its own vmcnt(0) at the branch join, which serialises the gathers (round 6: 59 -> ? us at config 2)
    constexpr int NW = SEL_THREADS / WAVE, CB3 = 8;
    for (int j0 = w; j0 < K3p; j0 += NW * CB3) {
      int64_t rowv[CB3];
#pragma unroll
      for (int i = 0; i < CB3; ++i) {
        const int j = j0 + NW * i;
        rowv[i] = (int64_t)(sh.sel[ord2[j < K3p ? j : K3p - 1]] & ROW_MASK);
      }
      if (a.remap)
#pragma unroll
        for (int i = 0; i < CB3; ++i) rowv[i] = a.remap[rowv[i]];
      int4 raw[CB3];
      double nrm[CB3];
#pragma unroll
      for (int i = 0; i < CB3; ++i) {
        raw[i] = phase3_load(a.x8 + rowv[i] * DIM);
        nrm[i] = a.norms[rowv[i]];
      }
#pragma unroll
      for (int i = 0; i < CB3; ++i) {
        const int j = j0 + NW * i;
        const double c = phase3_from(qv, raw[i], nrm[i]);
        if (j < K3p && l == 0) sh.s3[ord2[j]] = c;
      }
    }
  }
  __syncthreads();
  // gather s3 in Phase-II order, stable sort desc
  double* s3o = sh.s3o;
  for (int i = tid; i < K3p; i += SEL_THREADS) s3o[i] = sh.s3[ord2[i]];
  __syncthreads();
  stable_desc_order(s3o, K3p, sh);
  const int m = a.k < K3p ? a.k : K3p;
  for (int i = tid; i < a.kout; i += SEL_THREADS) {
    const int64_t o = (int64_t)qi * a.kout + i;
    if (i < m) {
      const int r = ord2[sh.sidx[i]];
      const uint64_t key = sh.sel[r];
      a.out_rows[o] = (int64_t)(key & ROW_MASK) + a.row_offset;
      a.out_dist[o] = (int32_t)(key >> KEY_ROW_BITS);
      a.out_s2[o] = sh.s2[r];
      a.out_s3[o] = sh.s3[r];
      if (a.out_src) a.out_src[o] = sh.pay[r];
    } else {
      a.out_rows[o] = -1;
      a.out_dist[o] = DIST_NONE;
      a.out_s2[o] = __builtin_nan("");
      a.out_s3[o] = __builtin_nan("");
      if (a.out_src) a.out_src[o] = -1;
    }
  }
  if (tid == 0) a.out_count[qi] = m;
}

// Per-query lists of the scan: nlp chunk lists [nq][nlp][K], optionally followed by one
// more list per query from a separate [nq][K] array (the matrix-core scan's suffix list,
// whose rows all follow the prefix lists' rows).
struct ScanKeys {
  const uint64_t* lists;
  const uint64_t* suffix;
  int nlpK;
  __device__ uint64_t operator[](int i) const { return i < nlpK ? lists[i] : suffix[i - nlpK]; }
};

// Phase II (:283-293) of the Kp candidates sh.sel[0..Kp) -> sh.s2, one candidate per lane.  The score is
// a sum of 256 nibble terms: for nibble p of the packed code (dims 4p..4p+3, MSB first) and its value v,
// T[p][v] = sum_b (bit b of v ? q[4p+b] : -q[4p+b]) -- exact in float64, like every partial sum of the
// reference's float32 x +-1 products -- so s2 = sum_p T[p][v_p] is the same exact value as the wave-wide
// ddot of phase2_dot, with 256 LDS lookups per candidate instead of 1024 products spread over a wave.
// The tables cover QT_NIB nibbles at a time (16 KiB of LDS: four workgroups of the small instance per CU).
constexpr int QT_NIB = 128;
template <class SH>
__device__ void phase2_nibble_tables(const float* __restrict__ q, const uint8_t* __restrict__ codes,
                                     const int64_t* __restrict__ remap, int Kp, SH& sh, double* qtab) {
  constexpr int NW = SEL_THREADS / WAVE;
  const int tid = threadIdx.x, w = tid / WAVE, l = lane_id();
  for (int jb = 0; jb < Kp; jb += SEL_THREADS) {  // candidates jb + 4 l + w (all of them when Kp <= 256)
    const int j = jb + NW * l + w;
    const bool live = j < Kp;
    int64_t row = (int64_t)(sh.sel[live ? j : 0] & ROW_MASK);
    if (remap) row = remap[row];
    double acc = 0.0;
    for (int half = 0; half < 256 / QT_NIB; ++half) {
      // this half's code bytes of the lane's row (bytes 64 half .. +63), loaded before the table build
      uint4 cw[4];
      const uint4* src = reinterpret_cast<const uint4*>(codes + row * (DIM / 8) + half * (QT_NIB / 2));
#pragma unroll
      for (int i = 0; i < 4; ++i) cw[i] = src[i];
      __syncthreads();  // (the previous half's lookups are done)
      for (int e = tid; e < QT_NIB * 16; e += SEL_THREADS) {
        const int p = e >> 4, v = e & 15, d0 = 4 * (half * QT_NIB + p);
        double t = 0.0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const double x = (double)q[d0 + b];
          t += ((v >> (3 - b)) & 1) ? x : -x;
        }
        qtab[e] = t;
      }
      __syncthreads();
      if (live) {
        const uint32_t wd[16] = {cw[0].x, cw[0].y, cw[0].z, cw[0].w, cw[1].x, cw[1].y, cw[1].z, cw[1].w,
                                 cw[2].x, cw[2].y, cw[2].z, cw[2].w, cw[3].x, cw[3].y, cw[3].z, cw[3].w};
#pragma unroll
        for (int k = 0; k < 16; ++k) {
#pragma unroll
          for (int c = 0; c < 4; ++c) {  // byte 4k + c (little-endian in the dword): nibbles 2(4k+c), +1
            const uint32_t byte = (wd[k] >> (8 * c)) & 0xffu;
            const int pb = 2 * (4 * k + c);
            acc += qtab[pb * 16 + (byte >> 4)];
            acc += qtab[(pb + 1) * 16 + (byte & 15)];
          }
        }
      }
    }
    if (live) sh.s2[j] = acc;
  }
  __syncthreads();
}

// mode: 0 = full 3-phase; 1 = Phase I only; 2 = shard (all Kp candidates, s2 + s3, Phase-I order)
template <class SH>
// (the small instance at 4 waves per SIMD: every query of a 1024-query batch resident at once)
__global__ __launch_bounds__(SEL_THREADS, SH::kKM <= KSMALL ? 4 : 1) void select_rescore_kernel(
    const uint64_t* __restrict__ lists, int nlp, const uint64_t* __restrict__ suffix, int K,
    const uint8_t* __restrict__ codes, const int8_t* __restrict__ x8, const double* __restrict__ norms,
    const float* __restrict__ qf, int mode, FinishArgs fa) {
  __shared__ SH sh;
  const int qi = blockIdx.x;
  const int tid = threadIdx.x, w = tid / WAVE, l = lane_id();
  const ScanKeys Lq{lists + (int64_t)qi * nlp * K, suffix ? suffix + (int64_t)qi * K : nullptr, nlp * K};
  int Kp;
  if (nlp == 0 && suffix) {
    // the matrix-core scan's suffix stage left one list, already the exact top-K in FAISS (dist, row)
    // order with KEY_NONE padding after its valid prefix: taken as is
    const uint64_t* sq = suffix + (int64_t)qi * K;
    if (tid == 0) sh.misc[0] = 0;
    __syncthreads();
    int valid = 0;
    for (int i = tid; i < K; i += SEL_THREADS) {
      const uint64_t key = sq[i];
      sh.sel[i] = key;
      sh.pay[i] = i;
      valid += key != KEY_NONE ? 1 : 0;
    }
    if (valid) atomicAdd(&sh.misc[0], valid);
    __syncthreads();
    Kp = sh.misc[0];
  } else {
    Kp = select_topk(Lq, nlp + (suffix ? 1 : 0), K, sh);
  }
  if (mode == 1) {
    for (int i = tid; i < fa.kout; i += SEL_THREADS) {
      const int64_t o = (int64_t)qi * fa.kout + i;
      if (i < Kp) {
        fa.out_rows[o] = (int64_t)(sh.sel[i] & ROW_MASK) + fa.row_offset;
        fa.out_dist[o] = (int32_t)(sh.sel[i] >> KEY_ROW_BITS);
      } else {
        fa.out_rows[o] = -1;
        fa.out_dist[o] = DIST_NONE;
      }
    }
    if (tid == 0 && fa.out_count) fa.out_count[qi] = Kp;
    return;
  }
#ifdef VRQ_FIN_BISECT  // timing-only probe builds (wrong results): 1 = stop after the selection
  if (VRQ_FIN_BISECT == 1) return;
#endif
  // Phase II for all Kp candidates (float64, :283-293)
  const float* q = qf + (int64_t)qi * DIM;
  __shared__ double qtab[QT_NIB * 16];
  phase2_nibble_tables(q, codes, fa.remap, Kp, sh, qtab);
  if (mode == 2) {
    float qv[DPL];
    load_q(qv, q);
    for (int j = w; j < Kp; j += SEL_THREADS / WAVE) {
      uint64_t row = sh.sel[j] & ROW_MASK;
      if (fa.remap) row = (uint64_t)fa.remap[row];
      const double c = phase3_cos(qv, x8 + row * DIM, norms[row]);
      if (l == 0) sh.s3[j] = c;
    }
    __syncthreads();
    for (int i = tid; i < fa.kout; i += SEL_THREADS) {
      const int64_t o = (int64_t)qi * fa.kout + i;
      if (i < Kp) {
        fa.out_rows[o] = (int64_t)(sh.sel[i] & ROW_MASK) + fa.row_offset;
        fa.out_dist[o] = (int32_t)(sh.sel[i] >> KEY_ROW_BITS);
        fa.out_s2[o] = sh.s2[i];
        fa.out_s3[o] = sh.s3[i];
      } else {
        fa.out_rows[o] = -1;
        fa.out_dist[o] = DIST_NONE;
        fa.out_s2[o] = __builtin_nan("");
        fa.out_s3[o] = __builtin_nan("");
      }
    }
    if (tid == 0) fa.out_count[qi] = Kp;
    return;
  }
  __syncthreads();
#ifdef VRQ_FIN_BISECT  // 2 = stop after Phase II
  if (VRQ_FIN_BISECT == 2) return;
#endif
  FinishArgs a = fa;
  a.q = q;
  finish_query(Kp, false, a, qi, sh);
}

// Shard merge: the lists are the shards' (dist, global row) candidates (VRQ_SEARCH_SHARD
// outputs stacked [S][nq][K]); the payload carried to the finish step is s2/s3.
struct ShardKeys {
  const int32_t* counts;
  const int64_t* rows;
  const int32_t* dist;
  int nq, qi, K;
  __device__ uint64_t operator[](int i) const {
    const int s = i / K, p = i - s * K;
    const int64_t src = ((int64_t)s * nq + qi) * K + p;
    if (p >= counts[(int64_t)s * nq + qi] || rows[src] < 0) return KEY_NONE;
    return ((uint64_t)(uint32_t)dist[src] << KEY_ROW_BITS) | ((uint64_t)rows[src] & ROW_MASK);
  }
};

template <class SH>
__global__ __launch_bounds__(SEL_THREADS) void merge_shards_kernel(int S, int K, const int32_t* __restrict__ counts,
                                                                   const int64_t* __restrict__ rows,
                                                                   const int32_t* __restrict__ dist,
                                                                   const double* __restrict__ s2,
                                                                   const double* __restrict__ s3, int nq,
                                                                   FinishArgs fa) {
  __shared__ SH sh;
  const int qi = blockIdx.x;
  const int tid = threadIdx.x;
  const ShardKeys L{counts, rows, dist, nq, qi, K};
  const int Kp = select_topk(L, S, K, sh);
  for (int j = tid; j < Kp; j += SEL_THREADS) {
    const int i = sh.pay[j];
    const int s = i / K, p = i - s * K;
    const int64_t src = ((int64_t)s * nq + qi) * K + p;
    sh.s2[j] = s2[src];
    sh.s3[j] = s3[src];
  }
  __syncthreads();
  FinishArgs a = fa;
  a.row_offset = 0;
  finish_query(Kp, true, a, qi, sh);
}

// Stand-alone candidate rescoring: one wave per (query, candidate).
__global__ __launch_bounds__(256) void rescore_kernel(int which, const float* __restrict__ qf, int nq,
                                                      const uint8_t* __restrict__ codes,
                                                      const int8_t* __restrict__ x8,
                                                      const double* __restrict__ norms, int64_t n,
                                                      const int64_t* __restrict__ cand, int ncand,
                                                      double* __restrict__ out) {
  const int64_t gw = ((int64_t)blockIdx.x * 256 + threadIdx.x) / WAVE;
  if (gw >= (int64_t)nq * ncand) return;
  const int qi = (int)(gw / ncand);
  const int64_t row = cand[gw];
  if (row < 0 || row >= n) {
    if (lane_id() == 0) out[gw] = __builtin_nan("");
    return;
  }
  float qv[DPL];
  load_q(qv, qf + (int64_t)qi * DIM);
  const double v = which == 0 ? phase2_dot(qv, codes + row * (DIM / 8)) : phase3_cos(qv, x8 + row * DIM, norms[row]);
  if (lane_id() == 0) out[gw] = v;
}

// launch the small-LDS instance when the shape fits it
static int launch_select(hipStream_t s, int nq, const uint64_t* lists, int nlp, const uint64_t* suffix, int K,
                         const uint8_t* codes, const int8_t* x8, const double* norms, const float* qf, int mode,
                         const FinishArgs& fa) {
  const int nl = nlp + (suffix ? 1 : 0);
  if (K <= KSMALL && nl <= LSMALL)
    hipLaunchKernelGGL(select_rescore_kernel<SelSmall>, dim3(nq), dim3(SEL_THREADS), 0, s, lists, nlp, suffix, K,
                       codes, x8, norms, qf, mode, fa);
  else
    hipLaunchKernelGGL(select_rescore_kernel<SelBig>, dim3(nq), dim3(SEL_THREADS), 0, s, lists, nlp, suffix, K,
                       codes, x8, norms, qf, mode, fa);
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

}  // namespace vrq

using namespace vrq;

extern "C" {

size_t vrq_search3_workspace_size(int64_t n, int32_t dim, int32_t nq, int32_t K) {
  if (n < 1 || nq < 1 || K < 1 || dim != DIM) return 0;
  ScanPlan p;
  if (scan_plan(n, dim / 8, nq, K, &p) != VRQ_OK) return 0;
  MfmaPlan mp;
  if (K <= kMfmaMaxK && n >= kMfmaMinRows && mfma_plan(n, nq, K, &mp) == VRQ_OK)
    return mp.bytes > p.list_bytes ? mp.bytes : p.list_bytes;
  return p.list_bytes;
}

size_t vrq_hamming_topk_workspace_size(int64_t n, int32_t code_bytes, int32_t nq, int32_t k) {
  if (n < 1 || nq < 1 || k < 1) return 0;
  ScanPlan p;
  if (scan_plan(n, code_bytes, nq, k, &p) != VRQ_OK) return 0;
  MfmaPlan mp;
  if (code_bytes == 128 && mfma_use(n, nq, k, 0) && mfma_plan(n, nq, k, &mp) == VRQ_OK)
    return mp.bytes > p.list_bytes ? mp.bytes : p.list_bytes;
  return p.list_bytes;
}

static int fill_empty(int32_t nq, int32_t kout, int32_t* out_count, int64_t* out_rows, int32_t* out_dist,
                      double* out_s2, double* out_s3, hipStream_t s) {
  // n == 0 or K == 0: no candidates (CohereEnhancedVectorDB.py:247-249, :277-279)
  if (out_count && hipMemsetAsync(out_count, 0, sizeof(int32_t) * nq, s) != hipSuccess) return VRQ_EHIP;
  const size_t m = (size_t)nq * kout;
  if (m == 0) return VRQ_OK;
  if (out_rows && hipMemsetAsync(out_rows, 0xff, sizeof(int64_t) * m, s) != hipSuccess) return VRQ_EHIP;   // -1
  if (out_dist && hipMemsetAsync(out_dist, 0x7f, sizeof(int32_t) * m, s) != hipSuccess) return VRQ_EHIP;   // ~INT_MAX
  if (out_s2 && hipMemsetAsync(out_s2, 0xff, sizeof(double) * m, s) != hipSuccess) return VRQ_EHIP;       // NaN
  if (out_s3 && hipMemsetAsync(out_s3, 0xff, sizeof(double) * m, s) != hipSuccess) return VRQ_EHIP;
  return VRQ_OK;
}

int vrq_hamming_topk(const uint8_t* codes, int64_t n, int32_t code_bytes, int64_t row_offset,
                     const uint8_t* queries, int32_t nq, int32_t k, int32_t* out_dist, int64_t* out_rows,
                     void* workspace, size_t workspace_bytes, void* stream) {
  VRQ_CHECK_ARG(n >= 0 && nq >= 0 && k >= 0 && out_dist && out_rows);
  hipStream_t s = (hipStream_t)stream;
  if (nq == 0) return VRQ_OK;
  if (n == 0 || k == 0) return fill_empty(nq, k, nullptr, out_rows, out_dist, nullptr, nullptr, s);
  VRQ_CHECK_ARG(codes && queries && workspace);
  FinishArgs fa{};
  fa.row_offset = row_offset;
  fa.out_rows = out_rows;
  fa.out_dist = out_dist;
  fa.kout = k;
  uint64_t* lists = (uint64_t*)workspace;
  if (code_bytes == 128 && mfma_use(n, nq, k, 0)) {
    MfmaPlan mp;
    int rc = mfma_plan(n, nq, k, &mp);
    if (rc != VRQ_OK) return rc;
    if (workspace_bytes < mp.bytes) return VRQ_EWORKSPACE;
    rc = mfma_scan_launch(mp, codes, n, queries, nq, k, (uint8_t*)workspace, s, 0);
    if (rc != VRQ_OK) return rc;
    return launch_select(s, nq, lists, 0, (const uint64_t*)((uint8_t*)workspace + mp.off_suffix), k, nullptr,
                         nullptr, nullptr, nullptr, 1, fa);
  }
  ScanPlan p;
  int rc = scan_plan(n, code_bytes, nq, k, &p);
  if (rc != VRQ_OK) return rc;
  if (workspace_bytes < p.list_bytes) return VRQ_EWORKSPACE;
  if (p.nchunks > MAX_LISTS) return VRQ_EUNSUPPORTED;
  rc = scan_launch(p, codes, n, code_bytes, queries, nq, k, lists, s);
  if (rc != VRQ_OK) return rc;
  return launch_select(s, nq, lists, p.nchunks, nullptr, k, nullptr, nullptr, nullptr, nullptr, 1, fa);
}

int vrq_search3_scan(const uint8_t* codes, int64_t n, int32_t dim, const uint8_t* qb, int32_t nq, int32_t K,
                     int32_t flags, void* workspace, size_t workspace_bytes, void* stream) {
  VRQ_CHECK_ARG(n >= 0 && nq >= 0 && K >= 0);
  if (dim != DIM) return VRQ_EUNSUPPORTED;
  if (K > KMAX) return VRQ_EUNSUPPORTED;
  if (nq == 0 || n == 0 || K == 0) return VRQ_OK;
  VRQ_CHECK_ARG(codes && qb && workspace);
  if (mfma_use(n, nq, K, flags)) {
    MfmaPlan mp;
    const int rc = mfma_plan(n, nq, K, &mp);
    if (rc != VRQ_OK) return rc;
    if (workspace_bytes < mp.bytes) return VRQ_EWORKSPACE;
    return mfma_scan_launch(mp, codes, n, qb, nq, K, (uint8_t*)workspace, (hipStream_t)stream, flags);
  }
  ScanPlan p;
  int rc = scan_plan(n, dim / 8, nq, K, &p);
  if (rc != VRQ_OK) return rc;
  if (workspace_bytes < p.list_bytes) return VRQ_EWORKSPACE;
  if (p.nchunks > MAX_LISTS) return VRQ_EUNSUPPORTED;
  return scan_launch(p, codes, n, dim / 8, qb, nq, K, (uint64_t*)workspace, (hipStream_t)stream);
}

int vrq_search3_finish(const uint8_t* codes, const int8_t* x8, const double* norms, const int64_t* rescore_row,
                       int64_t n, int32_t dim, int64_t row_offset, const float* qf, int32_t nq, int32_t k, int32_t K,
                       int32_t K3, int32_t flags, int32_t* out_count, int64_t* out_rows, int32_t* out_dist,
                       double* out_binary, double* out_cosine, const void* workspace, size_t workspace_bytes,
                       void* stream) {
  VRQ_CHECK_ARG(n >= 0 && nq >= 0 && k >= 0 && K >= 0 && K3 >= 0);
  VRQ_CHECK_ARG(out_count && out_rows && out_dist);
  if (dim != DIM) return VRQ_EUNSUPPORTED;
  if (K > KMAX) return VRQ_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const int mode = (flags & VRQ_SEARCH_PHASE1_ONLY) ? 1 : (flags & VRQ_SEARCH_SHARD) ? 2 : 0;
  const int kout = mode == 0 ? k : K;
  if (nq == 0) return VRQ_OK;
  if (mode != 1) VRQ_CHECK_ARG(out_binary && out_cosine);
  if (n == 0 || K == 0 || (mode == 0 && k == 0))
    return fill_empty(nq, kout, out_count, out_rows, out_dist, out_binary, out_cosine, s);
  VRQ_CHECK_ARG(codes && workspace);
  if (mode != 1) VRQ_CHECK_ARG(qf && x8 && norms);
  int nlp;
  const uint64_t* suffix = nullptr;
  if (mfma_use(n, nq, K, flags)) {
    MfmaPlan mp;
    const int rc = mfma_plan(n, nq, K, &mp);
    if (rc != VRQ_OK) return rc;
    if (workspace_bytes < mp.bytes) return VRQ_EWORKSPACE;
    nlp = 0;  // the matrix-core scan leaves one sorted list per query
    suffix = (const uint64_t*)((const uint8_t*)workspace + mp.off_suffix);
  } else {
    ScanPlan p;
    const int rc = scan_plan(n, dim / 8, nq, K, &p);
    if (rc != VRQ_OK) return rc;
    if (workspace_bytes < p.list_bytes) return VRQ_EWORKSPACE;
    nlp = p.nchunks;
  }
  FinishArgs fa{};
  fa.x8 = x8;
  fa.norms = norms;
  fa.remap = rescore_row;
  fa.row_offset = row_offset;
  fa.k = k;
  fa.K3 = K3;
  fa.out_count = out_count;
  fa.out_rows = out_rows;
  fa.out_dist = out_dist;
  fa.out_s2 = out_binary;
  fa.out_s3 = out_cosine;
  fa.kout = kout;
  return launch_select(s, nq, (const uint64_t*)workspace, nlp, suffix, K, codes, x8, norms, qf, mode, fa);
}

int vrq_search3(const uint8_t* codes, const int8_t* x8, const double* norms, const int64_t* rescore_row,
                int64_t n, int32_t dim, int64_t row_offset, const float* qf, const uint8_t* qb, int32_t nq, int32_t k,
                int32_t K, int32_t K3, int32_t flags, int32_t* out_count, int64_t* out_rows, int32_t* out_dist,
                double* out_binary, double* out_cosine, void* workspace, size_t workspace_bytes, void* stream) {
  VRQ_CHECK_ARG(n >= 0 && nq >= 0 && k >= 0 && K >= 0 && K3 >= 0);
  const int mode = (flags & VRQ_SEARCH_PHASE1_ONLY) ? 1 : (flags & VRQ_SEARCH_SHARD) ? 2 : 0;
  const bool empty = n == 0 || K == 0 || (mode == 0 && k == 0);
  if (!empty && nq > 0) {
    const int rc = vrq_search3_scan(codes, n, dim, qb, nq, K, flags, workspace, workspace_bytes, stream);
    if (rc != VRQ_OK) return rc;
  }
  return vrq_search3_finish(codes, x8, norms, rescore_row, n, dim, row_offset, qf, nq, k, K, K3, flags, out_count,
                            out_rows, out_dist, out_binary, out_cosine, workspace, workspace_bytes, stream);
}

int vrq_scan_kind(int64_t n, int32_t dim, int32_t nq, int32_t K, int32_t flags, int64_t* prefix_rows) {
  if (n < 1 || nq < 1 || K < 1) return VRQ_EINVAL;
  if (dim != DIM || K > KMAX) return VRQ_EUNSUPPORTED;
  if (mfma_use(n, nq, K, flags)) {
    MfmaPlan mp;
    const int rc = mfma_plan(n, nq, K, &mp);
    if (rc != VRQ_OK) return rc;
    if (prefix_rows) *prefix_rows = 0;  // every row goes through the matrix-core pass
    return VRQ_SCAN_KIND_MFMA;
  }
  ScanPlan p;
  const int rc = scan_plan(n, dim / 8, nq, K, &p);
  if (rc != VRQ_OK) return rc;
  if (prefix_rows) *prefix_rows = n;
  return VRQ_SCAN_KIND_VALU;
}

int vrq_scan_plan(int64_t n, int32_t dim, int32_t nq, int32_t K, int32_t flags, int64_t* info) {
  if (!info || n < 1 || nq < 1 || K < 1) return VRQ_EINVAL;
  if (dim != DIM || K > KMAX) return VRQ_EUNSUPPORTED;
  if (!mfma_use(n, nq, K, flags)) return VRQ_EUNSUPPORTED;
  MfmaPlan p;
  const int rc = mfma_plan(n, nq, K, &p);
  if (rc != VRQ_OK) return rc;
  info[0] = p.rows ? 1 : p.swap ? 2 : 0;
  info[1] = p.mb;
  info[2] = p.chunk_rows;
  info[3] = p.nchunks;
  info[4] = p.capc;
  info[5] = (int64_t)p.off_cand;
  info[6] = (int64_t)p.off_cnt;
  info[7] = (int64_t)p.off_tau;
  info[8] = p.sample;
  info[9] = p.j;
  info[10] = (int64_t)p.off_suffix;
  info[11] = (int64_t)p.bytes;
  return VRQ_OK;
}

int vrq_scan_sample_plan(int64_t n, int32_t dim, int32_t nq, int32_t K, int32_t flags, int64_t* info) {
  if (!info || n < 1 || nq < 1 || K < 1) return VRQ_EINVAL;
  if (dim != DIM || K > KMAX) return VRQ_EUNSUPPORTED;
  if (!mfma_use(n, nq, K, flags)) return VRQ_EUNSUPPORTED;
  MfmaPlan p;
  const int rc = mfma_plan(n, nq, K, &p);
  if (rc != VRQ_OK) return rc;
  info[0] = p.rows_sample;
  info[1] = p.sample_chunks;
  info[2] = p.sample_chunk_rows;
  info[3] = p.sample_stride;
  info[4] = p.sample_tile_stride;
  info[5] = p.dvcols;
  return VRQ_OK;
}

int vrq_merge_shards(int32_t nshards, int32_t nq, int32_t K, const int32_t* counts, const int64_t* rows,
                     const int32_t* dist, const double* s2, const double* s3, int32_t k, int32_t K3,
                     int32_t* out_count, int64_t* out_rows, int32_t* out_dist, double* out_binary,
                     double* out_cosine, int32_t* out_src, void* stream) {
  VRQ_CHECK_ARG(nshards >= 1 && nq >= 0 && K >= 0 && k >= 0 && K3 >= 0);
  VRQ_CHECK_ARG(out_count && out_rows && out_dist && out_binary && out_cosine);
  if (K > KMAX || nshards > MAX_LISTS) return VRQ_EUNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  if (nq == 0) return VRQ_OK;
  if (K == 0 || k == 0) return fill_empty(nq, k, out_count, out_rows, out_dist, out_binary, out_cosine, s);
  VRQ_CHECK_ARG(counts && rows && dist && s2 && s3);
  FinishArgs fa{};
  fa.k = k;
  fa.K3 = K3;
  fa.out_count = out_count;
  fa.out_rows = out_rows;
  fa.out_dist = out_dist;
  fa.out_s2 = out_binary;
  fa.out_s3 = out_cosine;
  fa.out_src = out_src;
  fa.kout = k;
  if (K <= KSMALL && nshards <= LSMALL)
    hipLaunchKernelGGL(merge_shards_kernel<SelSmall>, dim3(nq), dim3(SEL_THREADS), 0, s, nshards, K, counts, rows,
                       dist, s2, s3, nq, fa);
  else
    hipLaunchKernelGGL(merge_shards_kernel<SelBig>, dim3(nq), dim3(SEL_THREADS), 0, s, nshards, K, counts, rows,
                       dist, s2, s3, nq, fa);
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

int vrq_rescore_binary(const float* qf, int32_t nq, int32_t dim, const uint8_t* codes, int64_t n,
                       const int64_t* cand_rows, int32_t ncand, double* out, void* stream) {
  VRQ_CHECK_ARG(nq >= 0 && ncand >= 0 && n >= 0);
  if (dim != DIM) return VRQ_EUNSUPPORTED;
  const int64_t waves = (int64_t)nq * ncand;
  if (waves == 0) return VRQ_OK;
  VRQ_CHECK_ARG(qf && codes && cand_rows && out);
  hipLaunchKernelGGL(rescore_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream, 0, qf,
                     nq, codes, nullptr, nullptr, n, cand_rows, ncand, out);
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

int vrq_rescore_int8_cosine(const float* qf, int32_t nq, int32_t dim, const int8_t* x8, const double* norms,
                            int64_t n, const int64_t* cand_rows, int32_t ncand, double* out, void* stream) {
  VRQ_CHECK_ARG(nq >= 0 && ncand >= 0 && n >= 0);
  if (dim != DIM) return VRQ_EUNSUPPORTED;
  const int64_t waves = (int64_t)nq * ncand;
  if (waves == 0) return VRQ_OK;
  VRQ_CHECK_ARG(qf && x8 && norms && cand_rows && out);
  hipLaunchKernelGGL(rescore_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, (hipStream_t)stream, 1, qf,
                     nq, nullptr, x8, norms, n, cand_rows, ncand, out);
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

}  // extern "C"
