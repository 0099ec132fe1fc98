// gemm_topk.hip -- K5 (BASELINE config 5): exhaustive Phase-II or Phase-III scoring of a batch of
// queries against the WHOLE corpus on the matrix cores (v_mfma_i32_32x32x32_i8), with the top-k
// fused in: the nq x n score matrix is never stored.
//
// Reference scores (exact_scores.h, bit-identical to the fused search's):
//   VRQ_GEMM_BINARY       s = float(q . (2*unpackbits(code)-1)), float64   CohereEnhancedVectorDB.py:283-293
//   VRQ_GEMM_INT8_COSINE  s = float32(q . int8) / ||int8||, -inf if 0      CohereEnhancedVectorDB.py:302-318
// Result per query: the k rows with the largest s, ordered (s desc, row asc) -- the reference's
// stable sorted(..., reverse=True) (:296, :321) over the rows taken in index order.
//
// Method (exact for every input):
//  1. prep: q/S = a + rho (one int8 "piece", S = max|q|/127) and rho the exact residual.  Delta_q bounds |u - s'| over all rows, where u is the matrix-core value below and
//     s' the reference score in the same units (Phase III: s/S; Phase II: (s + sum q)/(2S)):
//       Phase III  Delta = ||rho||_2 (Cauchy-Schwarz; the score divides by ||x||_2) + f32 slack
//       Phase II   Delta = max(sum rho+, sum rho-) (x in {0,1}: <rho, x> lies between them) + f32 slack
//  2. sample pass (dense): u for every (query, row) of an evenly spread row sample, where
//     u = fl(A) [* fl(1/||x||)] and A = <a, x> is an exact i32 MFMA dot product
//     (x = the int8 row, or the code's bits expanded to 0/1 bytes).  Only the running max of u per
//     (query, sample chunk, lane row) leaves the kernel: 32 values per query and chunk, each the u
//     of a distinct sample row (the [nq, S] matrix is never written).
//  3. select: U = the k-th largest of those maxima (<= the k-th largest sample u), thr = U - 2 Delta
//     (rounded down).  k distinct sample rows have u >= U, so s' >= U - Delta, and every row of the
//     exact top-k -- ties with the k-th included -- has u >= thr.
//  4. main pass: every row with u >= thr is appended to a per-(query, chunk) candidate list.
//  5. finish: exact reference scores of the candidates, running top-k by (s desc, row asc).  A list
//     overflow (heavy ties) or fewer than min(k, n) candidates (zero-norm rows) sends the query to
//     the exact fallback: one workgroup scans every row.
//
// Work decomposition of the two matrix passes: one workgroup per CU and 256-query block; the int8
// pieces of its queries for all of d = 1024 sit in the accumulator file (8 waves of 32 queries, two per
// SIMD; Phase II ran 4 waves of 64 until round 6).  32-row tiles stream HBM -> LDS by LDS-DMA (pieces
// spread over the MFMA shadow).  Phase III reads the int8 rows as B directly (XOR-swizzled image,
// conflict-free ds_read_b128); Phase II expands the packed bits into 0/1 bytes once per tile (shared by
// the eight waves) in a fixed k-permutation that the prep kernel applies to the queries as well.  The
// threshold test of tile t-1 runs in tile t's MFMA shadow.
#include <math.h>
#include <stdlib.h>

#include "exact_scores.h"
#include "mfma_common.h"
#include "vrq_internal.h"

namespace vrq {
namespace g5 {

// Matrix-pass layout: one workgroup per CU and 256-query block, the A fragments of its queries for
// all of d = 1024 in the accumulator file, one int8 piece per query (q/S = a + rho):
//   Phase III: 8 waves (two per SIMD) of 32 queries -- a SIMD's second wave keeps its matrix core busy
//              while the first issues its threshold tests and LDS-DMA pieces (main pass 8.8 vs 9.5 ms
//              for 4 waves of 64 at 10M x 1024, nq = 1024, round 3);
//   Phase II:  the same since round 6 (round 5: 4 waves of 64 queries, each B fragment feeding both
//              M-blocks, one wave per SIMD: the matrix cores 0.57 busy at 2.36 GHz).
// One piece (vs q/S = a + b/256 + rho) halves the MFMA work and doubles the corpus-byte reuse per
// query at a ~4x wider threshold margin (~2K exact rescorings per query at 10M rows): 29.3 vs 40.6 ms
// per 10M batch, both phases (round 2).
constexpr int GQB = 256;  // queries per workgroup
// Phase II runs the Phase-III layout (round 6): 8 waves of 32 queries, two per SIMD, each expanding half as
// many code dwords per tile as the round-5 4-wave layout, waves 0-3 issuing the tile's DMA.  The SIMD's
// second wave covers the waits that idled the matrix core (main pass 7.46 -> 6.8-7.1 ms at 10M x 1024,
// profiles/r6_c5_p2w8_ab.jsonl).  VRQ_G5_P2W8=0 (A/B builds) restores 4 waves of 64 queries.
#ifndef VRQ_G5_P2W8
#define VRQ_G5_P2W8 1
#endif
template <int PH>
struct KShape {
  static constexpr bool P3 = PH != VRQ_GEMM_BINARY;
  static constexpr int W = (P3 || VRQ_G5_P2W8) ? 8 : 4, MB = (P3 || VRQ_G5_P2W8) ? 1 : 2, QW = 32 * MB,
                       NE = 16 * MB, RPW = 32 / W;
  static_assert(W * QW == GQB, "query block");
};
// planning target for the candidates per query (the sample size follows from it), and the
// per-(query, chunk) list capacity as a multiple of the hits the sample predicts
constexpr int FIN_CAP = 8192;
constexpr int CAP_MULT = 16;
// thresholded pass: a tile's hits (at most one per lane: the usual case) go to a per-wave LDS stage by
// wave-prefix positions (no atomic, no wait), drained into the per-(query, chunk) lists once per chunk
constexpr int STG5 = 1024;  // staged hit entries per wave (u32: query-in-wave << 26 | chunk row)
constexpr int64_t kMaxChunkRows = (int64_t(1) << 26) - 32;  // chunk rows fit the stage's 26-bit field
constexpr int GRT = 32;              // corpus rows per tile (one 32-column N-block)
constexpr int GKS = 32;              // k-steps of 32 dims (d = 1024)
constexpr int T3 = GRT * 1024;       // Phase-III tile: 32 int8 rows (32 KiB) ...
constexpr int T3N = T3 + GRT * 8;    // ... + their 32 f64 norms
constexpr int T2 = GRT * 128;        // Phase-II packed tile (4 KiB)
constexpr int U2 = GKS * 1024;       // Phase-II unpacked tile [k-step][lane][16 B] (32 KiB)
// tile schedule: B fragments read BA k-steps ahead; the LDS-DMA pieces of the tile AHEAD tiles
// ahead issue every DS k-steps from k-step 2 (round 3 sweeps of both moved nothing)
#ifndef VRQ_G5_BA  // (round 6, 8-wave Phase II: BA = 3 costs 0.45 ms (Phase II) and 0.55 ms (Phase III) per main
#define VRQ_G5_BA 2   // pass, profiles/r6_c5_ba3_ab.jsonl)
#endif
constexpr int BA = VRQ_G5_BA, DS = 3;

// main-pass chunks per (CU, query block): 4 keeps the query blocks that stream the same chunk
// within L2 reach of each other (PMC bytes 1.1x algorithmic vs 1.9x at 1, equal time; round 2)
constexpr int kChunkMult = 4;
constexpr int FB_BATCH = 1024;       // rows per batch of the exact fallback
constexpr int KMAX5 = 1024;          // k bound of the path
constexpr int64_t kMinSample = 32768;
constexpr int64_t kMaxSample = 1 << 21;
constexpr int QA_BYTES = 1024;       // per query: the int8 piece in fragment order

// Phase-II k-permutation inside a 32-dim k-step: fragment byte j = 4t + b of lane half h holds
// bit 8b + t + 4h of the little-endian code dword (so a dword of the fragment is (w >> (t+4h)) &
// 0x01010101, two VALU ops), i.e. packbits dim 8b + 7 - (t + 4h) of the step.
__host__ __device__ constexpr int ph2_pos(int dim_in_step) {
  const int b = dim_in_step >> 3, x = 7 - (dim_in_step & 7);  // byte, bit within the byte
  const int h = x >> 2, t = x & 3;
  return h * 16 + 4 * t + b;
}

__device__ __forceinline__ v16i mfma_i8(const v4i& a, const v4i& b, const v16i& c) {
  return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void lds_read64(double& d, uint32_t a) {
  asm volatile("ds_read_b64 %0, %1" : "=v"(d) : "v"(a) : "memory");
}
template <int OFF>
__device__ __forceinline__ void lds_read128_off(v4i& d, uint32_t a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF) : "memory");
}

// Monotone u32 image of a float for ASCENDING order; NaN -> 0 (below -inf).
__device__ __forceinline__ uint32_t fkey(float u) {
  const uint32_t b = __float_as_uint(u);
  if ((b & 0x7fffffffu) > 0x7f800000u) return 0u;
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
__device__ __forceinline__ double desc_key_inv(uint64_t key) {
  const uint64_t a = ~key;
  return __longlong_as_double((long long)((a & 0x8000000000000000ull) ? (a & 0x7fffffffffffffffull) : ~a));
}

// XCD-aware bijective block remap: consecutive logical blocks share one XCD's L2
__device__ __forceinline__ int xcd_logical(int b, int nb) {
  const int xcd = b & 7, slot = b >> 3, q8 = nb >> 3, r8 = nb & 7;
  return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
}

// ---------------------------------------------------------------------------------------------
// prep: one wave per (padded) query.  qa[q] = the piece a in fragment order (natural k order for
// Phase III, ph2_pos for Phase II); delta[q] = Delta_q in u units; (alpha[q], beta[q]) map a reference
// score s to u units (s' = alpha s + beta), for the raised threshold of the retry pass.
__global__ __launch_bounds__(256) void gemm_prep_kernel(int mode, const float* __restrict__ qf, int nq, int nq_pad,
                                                        int8_t* __restrict__ qa, double* __restrict__ delta,
                                                        double* __restrict__ alpha, double* __restrict__ beta,
                                                        const double* __restrict__ bounds) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), l = lane_id();
  if (q >= nq_pad) return;
  int8_t* o = qa + (int64_t)q * QA_BYTES;
  if (q >= nq) {  // padding queries: zero pieces (their thresholds never accept)
    reinterpret_cast<int4*>(o)[l] = make_int4(0, 0, 0, 0);
    if (l == 0) {
      delta[q] = 0.0;
      alpha[q] = 0.0;
      beta[q] = 0.0;
    }
    return;
  }
  float qv[DPL];
  load_q(qv, qf + (int64_t)q * DIM);
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < DPL; ++i) mx = fmaxf(mx, fabsf(qv[i]));
#pragma unroll
  for (int m = 1; m < WAVE; m <<= 1) mx = fmaxf(mx, __shfl_xor(mx, m, WAVE));
  // S = max|q| / 127 (the rounding of q/S in f64 is far inside the slack below)
  const double invS = mx > 0.f ? 127.0 / (double)mx : 1.0;
  double r2 = 0.0, rp = 0.0, rn = 0.0, q2 = 0.0, q1 = 0.0, qs = 0.0;
#pragma unroll
  for (int i = 0; i < DPL; ++i) {
    const double x = (double)qv[i] * invS;
    double a = rint(x);                     // |a| <= 127
    a = a > 127.0 ? 127.0 : (a < -127.0 ? -127.0 : a);
    const double rho = x - a;               // exact, |rho| <= 1/2
    r2 += rho * rho;
    rp += rho > 0.0 ? rho : 0.0;
    rn += rho < 0.0 ? -rho : 0.0;
    q2 += (double)qv[i] * (double)qv[i];
    q1 += fabs((double)qv[i]);
    qs += (double)qv[i];
    const int dim = DPL * l + i, s = dim >> 5;
    const int pos = s * 32 + (mode == VRQ_GEMM_BINARY ? ph2_pos(dim & 31) : (dim & 31));
    o[pos] = (int8_t)a;
  }
  r2 = wave_sum_f64(r2);
  rp = wave_sum_f64(rp);
  rn = wave_sum_f64(rn);
  q2 = wave_sum_f64(q2);
  q1 = wave_sum_f64(q1);
  qs = wave_sum_f64(qs);
  constexpr double SLACK = 1.0 / (1 << 20);  // >= 16 f32 ulps of every rounding on the u path
  if (l == 0) {
    double d;
    if (mode == VRQ_GEMM_BINARY) {
      // x in {0, 1}: u - s' = -<rho, x> lies in [-sum rho+, sum rho-], so |u - s'| <= max of the
      // two one-sided sums (about half of ||rho||_1)
      d = fmax(rp, rn) * (1.0 + SLACK) + SLACK * q1 * invS;
    } else if (mode == VRQ_GEMM_FLOAT_IP) {
      // u = s_r <a, b_r> against s' = <q/S, x_r> with x_r = s_r b_r + sigma_r (flat_ip_prepare):
      // |u - s'| <= ||rho|| ||s_r b_r|| + ||q/S|| ||sigma_r|| <= ||rho|| Bx + ||q/S|| Bsigma, and
      // |u| <= ||a|| Bx <= (||q/S|| + ||rho||) Bx scales the f32 slack
      const double qn = sqrt(q2) * invS, rn = sqrt(r2), bx = bounds[0], bs = bounds[1];
      d = (rn * bx + qn * bs) * (1.0 + SLACK) + SLACK * (qn + rn) * bx;
    } else {
      d = sqrt(r2) * (1.0 + SLACK) + SLACK * sqrt(q2) * invS;
    }
    delta[q] = d;
    // u units of a reference score s (s' = alpha s + beta): Phase II (s + sum q) / (2S), else s / S
    alpha[q] = mode == VRQ_GEMM_BINARY ? 0.5 * invS : invS;
    beta[q] = mode == VRQ_GEMM_BINARY ? 0.5 * invS * qs : 0.0;
  }
}

// ---------------------------------------------------------------------------------------------
// The matrix pass.  PH = VRQ_GEMM_BINARY / VRQ_GEMM_INT8_COSINE; DENSE = the sample pass (the max
// of u over each lane row's rows of the chunk -> dv[q][chunk * 32 + lane row]) else the thresholded
// pass (u >= thr[q] -> candidate lists).  Chunk c covers rows [c * chunk_stride, + chunk_rows).
// RETRY: the retry pass of launch_finish (same code; a separate symbol so kernel traces and counter
// summaries keep the main pass's per-launch figures apart from the retry's near-empty launch).
template <int PH, bool DENSE, bool RETRY = false>
__global__ __launch_bounds__(KShape<PH>::W * 64, 1) void gemm_topk_kernel(
    const uint8_t* __restrict__ src, const double* __restrict__ norms, int64_t n, const int8_t* __restrict__ qa,
    int nq, const float* __restrict__ thr, uint32_t* __restrict__ cand, int32_t* __restrict__ ccnt, int capc,
    int64_t chunk_rows, int64_t chunk_stride, int nchunks, int nqb, float* __restrict__ dv, int64_t dv_stride,
    const int32_t* __restrict__ qbflag) {
  constexpr bool P3 = PH == VRQ_GEMM_INT8_COSINE;
  constexpr int KW = KShape<PH>::W, KMB = KShape<PH>::MB, KQW = KShape<PH>::QW, KNE = KShape<PH>::NE;
  constexpr int RPW = KShape<PH>::RPW;               // Phase III: tile rows streamed per wave
  // Phase III: ring of 2 raw tiles (32 int8 rows + their norms), tile t+1 streamed in during tile t
  // (5 DMA pieces per wave: 4 rows + the norms).  Phase II: ring of 4 packed tiles, tile t+3 streamed in
  // during tile t (1 piece per wave), and the packed tile t+1 expanded into the unpacked ring (2 tiles).
  constexpr int NP = P3 ? 2 : 4;
  constexpr int PKT = P3 ? T3N : T2;                  // ring slot bytes
  constexpr int SMEM = NP * PKT + (P3 ? 0 : 2 * U2);
  constexpr int PPW = P3 ? RPW + 1 : 1;               // vector-memory instructions per wave per tile
  constexpr int AHEAD = NP - 1;                       // tiles the DMA runs ahead
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM];
  constexpr bool STAGE = !DENSE;
  // per-(query, this chunk) list lengths (one row per wave), then each wave's hit stage
  __shared__ int32_t lcnt[KW * KQW + (STAGE ? KW * STG5 : 0)];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = lane_id(), r = l & 31, h = l >> 5;
  const int L = xcd_logical(blockIdx.x, gridDim.x);
  const int chunk = L / nqb, qb = L - chunk * nqb;
  if (chunk >= nchunks) return;
  if (qbflag && qbflag[qb] == 0) return;  // retry pass: only query blocks holding a retried query
  const int64_t row0 = (int64_t)chunk * chunk_stride;
  const int64_t row1 = (row0 + chunk_rows < n) ? row0 + chunk_rows : n;
  if (row0 >= row1) return;
  const int nrows = (int)(row1 - row0);
  const int ntiles = (nrows + GRT - 1) / GRT;
  const uint32_t sm0 = lds_addr(smem);

  // ---- Tiles: tile t covers chunk rows [tstart(t), tstart(t) + 32).  The last tile of a chunk whose
  // length is not a multiple of 32 is shifted back to end at the chunk's end; its first rows (already
  // in the previous tile) are masked out, so every DMA reads a whole, in-bounds 32-row tile.  Only a
  // chunk shorter than 32 rows (tiny corpus) clamps rows instead.
  const bool tiny = nrows < GRT;
  auto tstart = [&](int t) { return tiny ? 0 : (t * GRT < nrows - GRT ? t * GRT : nrows - GRT); };
  auto lane_valid = [&](int t) {  // this lane's tile row r holds a row of tile t not seen before
    return tiny ? r < nrows : r >= t * GRT - tstart(t);
  };
  // ---- LDS-DMA of tile t (piece i of PPW per wave): a uniform base plus a per-lane offset.
  //   Phase III: tile row rr = 4w + i -> slots rr*64 + c', holding 16-B chunk c' ^ (rr & 15) of the
  //              row; piece 4 = the tile's 32 f64 norms (every wave loads the same 256 B, so the DMA
  //              count per wave is uniform).
  //   Phase II:  rows 8w..8w+7 -> slot rr*8 + c' holding chunk c' ^ ((rr >> 1) & 7).
  const int RB = P3 ? 1024 : 128;  // bytes per corpus row
  uint32_t loff[P3 ? RPW : 1];
  if constexpr (P3) {
#pragma unroll
    for (int i = 0; i < RPW; ++i) loff[i] = (uint32_t)(i * 1024 + ((l ^ ((RPW * w + i) & 15)) << 4));
  } else {
    const int rr = 8 * w + (l >> 3);
    loff[0] = (uint32_t)((l >> 3) * 128 + (((l & 7) ^ ((rr >> 1) & 7)) << 4));
  }
  // per-tile uniform DMA bases (computed once per tile, held in SGPRs); piece i adds lane offsets
  struct DmaTile {
    const uint8_t* gsrc;
    const uint8_t* gnrm;
    uint8_t* lds;
  };
  auto dma_tile = [&](int t, int slot_i) {  // whole tiles (not tiny)
    const int64_t tr0 = row0 + tstart(t);
    DmaTile d;
    d.gsrc = src + (tr0 + (P3 ? RPW : 8) * w) * RB;
    d.gnrm = reinterpret_cast<const uint8_t*>(norms + tr0);
    d.lds = smem + slot_i * PKT;
    return d;
  };
  constexpr bool P2W8 = !P3 && KW == 8;  // Phase II on 8 waves: the tile's 32 rows DMA'd by waves 0-3
  auto issue_piece = [&](const DmaTile& d, int i) {
    if (P2W8 && w >= 4) return;
    // (pointer arguments through locals: a compound expression here makes the host-side compile
    // silently drop the kernel's launch stub)
    if (P3 && i == RPW) {
      const uint8_t* g = d.gnrm + 4 * l;
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(d.lds + T3), 4, 0, 0);
      return;
    }
    const uint8_t* g = d.gsrc + loff[P3 ? i : 0];
    uint8_t* ld = d.lds + (P3 ? (RPW * w + i) * 1024 : w * 1024);
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)ld, 16, 0, 0);
  };
  auto issue_tiny = [&](int i) {  // the single tile of a chunk shorter than 32 rows: clamp rows
    if (P2W8 && w >= 4) return;
    if (P3 && i == RPW) {
      int64_t nr = row0 + (l >> 1);
      nr = nr < row1 ? nr : row1 - 1;
      const uint8_t* g = reinterpret_cast<const uint8_t*>(norms + nr) + 4 * (l & 1);
      __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + T3), 4, 0, 0);
      return;
    }
    const int rr = P3 ? RPW * w + i : 8 * w + (l >> 3);
    int64_t row = row0 + rr;
    row = row < row1 ? row : row1 - 1;
    const uint8_t* g = src + row * RB + (P3 ? ((l ^ (rr & 15)) << 4) : ((((l & 7) ^ ((rr >> 1) & 7))) << 4));
    __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)(smem + (P3 ? (RPW * w + i) * 1024 : w * 1024)),
                                     16, 0, 0);
  };
  // Phase II expansion: lane (r, h) of wave w takes code dwords 4c..4c+3 of tile row r, c = 2w + h
  // (k-steps 4c..4c+3), and writes both lane halves' fragments of each ([k-step][lane][16 B])
  // (8 waves: lane (r, h) of wave w takes code dwords 2c, 2c+1, c = 2w + h, i.e. half of 16-B chunk w)
  const int uc = 2 * w + h;
  constexpr int UD = P2W8 ? 2 : 4;  // code dwords a lane expands per tile
  const uint32_t usrc = (uint32_t)((r * 8 + ((P2W8 ? w : uc) ^ ((r >> 1) & 7))) * 16);
  auto unpack_frag = [&](const v4i& pv, int j, uint32_t ubw) {  // j = 2i + hh
    const int i = j >> 1, hh = j & 1;
    uint32_t wd;
    if constexpr (P2W8)
      wd = (uint32_t)(i == 0 ? (h ? pv.z : pv.x) : (h ? pv.w : pv.y));
    else
      wd = (uint32_t)(i == 0 ? pv.x : i == 1 ? pv.y : i == 2 ? pv.z : pv.w);
    v4i f;
    f.x = (int)((wd >> (4 * hh + 0)) & 0x01010101u);
    f.y = (int)((wd >> (4 * hh + 1)) & 0x01010101u);
    f.z = (int)((wd >> (4 * hh + 2)) & 0x01010101u);
    f.w = (int)((wd >> (4 * hh + 3)) & 0x01010101u);
    lds_write128(ubw + (uint32_t)(((UD * uc + i) * 64 + hh * 32 + r) * 16), f);
  };

  for (int t = 0; t < AHEAD && t < ntiles; ++t) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      if (tiny)
        issue_tiny(i);
      else
        issue_piece(dma_tile(t, t), i);
    }
  }

  // A fragments of this wave's M-blocks of 32 queries, all 32 k-steps -> accumulator file
  const int qbase = qb * GQB + w * KQW;
  v4i A[KMB][GKS];
#pragma unroll
  for (int j = 0; j < KMB; ++j) {
    const int8_t* qp = qa + (int64_t)(qbase + 32 * j + r) * QA_BYTES + h * 16;
#pragma unroll
    for (int s = 0; s < GKS; ++s) A[j][s] = *reinterpret_cast<const v4i*>(qp + s * 32);
  }
#pragma unroll
  for (int j = 0; j < KMB; ++j)
#pragma unroll
    for (int s = 0; s < GKS; ++s) asm volatile("" : "+a"(A[j][s]));
  // test e of a lane: M-block e >> 4, accumulator register g = e & 15 -> query row of the wave
  auto qrow = [&](int e) { return 32 * (e >> 4) + ((e & 3) + 8 * ((e >> 2) & 3) + 4 * h); };
  float th[KNE];
#pragma unroll
  for (int e = 0; e < KNE; ++e) th[e] = DENSE ? 0.f : thr[qbase + qrow(e)];
  // the thresholds land here, before the tile loop: the compiler's wait for a global load it still
  // sees in flight would otherwise sit at their first use INSIDE the loop as an s_waitcnt vmcnt(0),
  // which every tile then executes after issuing its LDS-DMA pieces (waiting for the next tile's DMA)
#pragma unroll
  for (int e = 0; e < KNE; ++e) asm volatile("" : "+v"(th[e]));
  // Phase-II thresholded pass: the accumulators start at -ceil(thr) (an integer seed per query: the
  // binary u is the integer dot), so a test is one integer max per accumulator register and the flush
  // re-derives the hit bits (acc >= 0) from the still-live accumulators
  constexpr bool SEED2 = !P3 && !DENSE;
  v16i seed[SEED2 ? KMB : 1];  // -ceil(thr) of each accumulator register's query, clamped
  if constexpr (SEED2) {
#pragma unroll
    for (int e = 0; e < KNE; ++e) {
      const float c = ceilf(th[e]);  // +-inf / huge thresholds: always / never a hit
      seed[e >> 4][e & 15] = c <= -1073741824.f ? 1073741824 : c >= 1073741824.f ? -1073741824 : -(int)c;
    }
  }
  int imax = INT32_MIN, iodd = 0;  // SEED2: running max of the seeded accumulators of the tested tile

  // Phase III: B fragment of k-step s for lane (r, h) = 16-B chunk 2s+h of tile row r, at slot
  // r*64 + ((2s+h) ^ (r & 15)) = r*64 + 16*(s>>3) + off[s&7]
  uint32_t boff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) boff[j] = (uint32_t)(((((2 * j) ^ (r & 14)) | (h ^ (r & 1))) << 4) + r * 1024);

  const uint32_t lc0 = lds_addr(lcnt + w * KQW);
  const uint32_t sg0 = lds_addr(lcnt + KW * KQW + (STAGE ? w * STG5 : 0));  // this wave's hit stage
  int nst = 0;  // staged entries (wave-uniform)
  if (!DENSE && l < KQW) lcnt[w * KQW + l] = 0;  // made visible by the first tile's barrier
  v16i acc[2][2] = {};   // [tile parity][M-block]
  // The sample pass keeps, per (lane, test), the running max of u over the chunk's rows of that lane.
  // Phase-III thresholded pass: test e of a tile leaves its hits as one wave mask (v_cmp into an SGPR
  // pair: cvt + fma + cmp per test, no per-lane bit assembly); the flush of tile t-2 ORs the 16 masks
  // on the scalar unit and builds per-lane bitmasks only for a tile with a hit.  (Measured at 10M x 1024,
  // nq = 1024, one box, two runs each: main pass 8.74 / 8.64 ms vs 8.82 / 8.92 ms for per-lane hit bits
  // and 8.99 / 8.95 ms for a recomputation from the still-live accumulators; round 3.)
  constexpr bool HWM = P3 && !DENSE;
  float ures[DENSE ? KNE : 1];
  uint64_t hmk[HWM ? KNE : 1] = {};
#pragma unroll
  for (int e = 0; e < (DENSE ? KNE : 1); ++e) ures[e] = DENSE ? __builtin_nanf("") : 0.f;
  float invc = 0.f, invp = 0.f, invpp = 0.f;  // Phase III 1/||x|| of tiles t, t-1, t-2 (NaN: zero norm or past the chunk)
  const v16i zero = {};
  const int64_t qstride = (int64_t)nchunks * capc;

  // u of test e from the accumulators of one tile (Phase III: NaN for rows without a score), minus
  // the query's threshold in the thresholded pass (one fma for Phase III)
  auto uval = [&](const v16i& a0, const v16i& a1, int e, float inv) {
    const int g = e & 15;
    const float u = (float)((e >> 4) ? a1[g] : a0[g]);
    if constexpr (DENSE)
      return P3 ? u * inv : u;
    else
      return P3 ? fmaf(u, inv, -th[e]) : u - th[e];
  };
  // hit of query-in-wave ql at chunk row cr -> its (query, chunk) list (position from this wave's LDS
  // counter; a list past capc keeps counting, which the finish kernel reads as an overflow)
  auto to_list = [&](int ql, int cr) {
    int pos;
    lds_add_rtn32(pos, lc0 + (uint32_t)(ql * 4), 1);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pos)::"memory");
    if (pos < capc) cand[(int64_t)(qbase + ql) * qstride + (int64_t)chunk * capc + pos] = (uint32_t)(row0 + cr);
  };
  // the staged entries -> lists (once per chunk, or when the stage is nearly full)
  auto drain = [&]() {
    for (int i0 = 0; i0 < nst; i0 += 64) {
      const int i = i0 + l;
      int e = 0;
      if (i < nst) lds_read32(e, sg0 + (uint32_t)(i * 4));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(e)::"memory");
      if (i < nst) to_list((int)((uint32_t)e >> 26), e & 0x3ffffff);
    }
    nst = 0;
  };
  // hits of tile tt (tested in the following tile's shadow) -> the stage; (a0, a1): tile tt's
  // accumulators (Phase II re-derives its hit bits from them)
  auto flush = [&](int tt, const v16i& a0, const v16i& a1) {
    const int lr = tstart(tt) + r;
    const bool ok = lane_valid(tt);
    if constexpr (!DENSE) {
      bool fl;
      if constexpr (HWM) {
        uint64_t any = 0;
#pragma unroll
        for (int e = 0; e < KNE; ++e) any |= hmk[e];
        fl = any != 0;
      } else {
        fl = __ballot(imax >= 0) != 0;
      }
      if (fl) {
        uint32_t m = 0;  // (hits: ~k * n / sample rows per query over the corpus)
        if constexpr (SEED2) {
          static_for<0, KNE>([&](auto E) {
            constexpr int e = decltype(E)::value;
            m |= (((e >> 4) ? a1 : a0)[e & 15] >= 0 ? 1u : 0u) << (KNE - 1 - e);
          });
        } else {
#pragma unroll
          for (int e = 0; e < KNE; ++e) {
            uint32_t b;
            asm volatile("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(b) : "v"(1u << (KNE - 1 - e)), "s"(hmk[e]));
            m |= b;
          }
        }
        if (!ok) m = 0;
        if (!__ballot((m & (m - 1)) != 0)) {
          // at most one hit per lane: one staged entry per hit lane at its rank among them
          const uint64_t lanes = __ballot(m != 0);
          if (m) {
            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(lanes >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)lanes, 0));
            const int ql = qrow(KNE - 1 - __builtin_ctz(m));
            lds_write32(sg0 + (uint32_t)((nst + below) * 4), (int)(((uint32_t)ql << 26) | (uint32_t)lr));
          }
          nst += __popcll(lanes);
          if (nst > STG5 - 64) drain();  // (rare: >= STG5 - 64 hits in one chunk)
        } else {
          while (m) {  // several hits in a lane: straight to the lists
            const int e = KNE - 1 - __builtin_ctz(m);
            m &= m - 1;
            to_list(qrow(e), lr);
          }
        }
      }
      imax = INT32_MIN;
    }
  };
  // Phase-II test of accumulator register e of the tested tile (pairs fold into one v_max3_i32)
  auto itest = [&](const v16i& a0, const v16i& a1, int e) {
    const int v = ((e >> 4) ? a1 : a0)[e & 15];
    if (e & 1)
      imax = max(imax, max(iodd, v));
    else
      iodd = v;
  };
  // the sample pass keeps, per (lane, test), the running max of u over the chunk's rows of that
  // lane (NaN: none yet; rows already seen in the previous tile, and Phase-III zero norms, are NaN
  // and drop out of the max); vp = this lane's row of the tested tile is new.  Phase-III thresholded
  // pass: the test's wave mask (NaN: no hit).
  auto test = [&](float u, int e, bool vp) {
    if constexpr (DENSE)
      ures[e] = fmaxf(ures[e], vp ? u : __builtin_nanf(""));
    else
      hmk[e] = __ballot(u >= 0.f);
  };

  if constexpr (!P3) {  // expand tile 0 before the loop (tile t+1 is expanded during tile t)
    wait_vm<0>();
    barrier_all();
    v4i pv;
    lds_read128(pv, sm0 + usrc);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pv)::"memory");
#pragma unroll
    for (int j = 0; j < 2 * UD; ++j) unpack_frag(pv, j, sm0 + (uint32_t)(NP * T2));
    wait_lgkm0();
  }

  int sl = 0;  // t % NP
  constexpr int NR = 4;  // B fragment ring (power of two > BA)
  static_assert(BA < NR, "B ring");
  auto tile = [&](auto PAR, auto FIRST, int t) {
    constexpr int p = decltype(PAR)::value;
    constexpr bool first = decltype(FIRST)::value;  // tile 0: no previous tile to test
    // The DMA of the tile needed now (Phase III: t; Phase II: t+1) landed; the INF tiles issued after
    // it may stay in flight (in the chunk's last tiles: wait for everything).  After the barrier every
    // wave's has, the expanded tile t is visible, and every wave is done reading the slots the DMA of
    // this tile overwrites.
    {
      constexpr int NEED = P3 ? 0 : 1, INF = AHEAD - 1 - NEED;
      if (t + NEED + INF < ntiles)
        wait_vm<INF * PPW>();
      else
        wait_vm<0>();
    }
    barrier_all();
    // tile t-2's hits: Phase II before the tile's first MFMA (its accumulators are acc[p] until then);
    // Phase III reads only its wave masks, so its flush sits at k-step FLS = 1, in the MFMA shadow
    constexpr int FLS = P3 && !DENSE ? 1 : -1;
    if (FLS < 0 && !DENSE && t >= 2) flush(t - 2, acc[p][0], acc[p][1]);
    const bool vprev = DENSE ? lane_valid(t - 1) : true;  // (the sample pass's test of tile t-1)
    const uint32_t slot = sm0 + (uint32_t)(sl * PKT);
    const bool dma = t + AHEAD < ntiles;
    const DmaTile dt = dma_tile(dma ? t + AHEAD : t, sl == 0 ? NP - 1 : sl - 1);
    const int sl1 = sl + 1 == NP ? 0 : sl + 1;                       // (t + 1) % NP
    double nv = 0.0;
    v4i pv = {};
    const uint32_t ubn = sm0 + (uint32_t)(NP * T2 + ((t + 1) & 1) * U2);  // Phase II: tile t+1 expanded here
    uint32_t badr[8];
    if constexpr (P3) {
      lds_read64(nv, slot + T3 + (uint32_t)(r * 8));
#pragma unroll
      for (int j = 0; j < 8; ++j) badr[j] = slot + boff[j];
    } else {
      badr[0] = sm0 + (uint32_t)(NP * T2 + (t & 1) * U2 + l * 16);
    }
    v4i ring[NR];
    auto readB = [&](auto S) {
      constexpr int s = decltype(S)::value;
      if constexpr (P3)
        lds_read128_off<(s >> 3) * 256>(ring[s & (NR - 1)], badr[s & 7]);
      else
        lds_read128_off<s * 1024>(ring[s & (NR - 1)], badr[0]);
    };
    static_for<0, BA>([&](auto S) { readB(S); });
    VRQ_SCHED_FENCE();
    static_for<0, GKS>([&](auto S) {
      constexpr int s = decltype(S)::value;
      if constexpr (s + BA < GKS) {
        readB(std::integral_constant<int, s + BA>{});
        // everything but the BA newest LDS operations is complete: B(s), and the norm (issued
        // before B(0)) / the packed Phase-II tile (issued in step 1, before B(1 + BA))
        asm volatile("s_waitcnt lgkmcnt(%3)" : "+v"(ring[s & (NR - 1)]), "+v"(nv), "+v"(pv) : "n"(BA) : "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(ring[s & (NR - 1)]) : "n"(GKS - 1 - s) : "memory");
      }
      if constexpr (SEED2) {  // tile starts at -ceil(thr) (Phase II: two M-blocks, one on 8 waves)
        acc[p][0] = mfma_i8(A[0][s], ring[s & (NR - 1)], s == 0 ? seed[0] : acc[p][0]);
        if constexpr (KMB == 2)
          acc[p][1] = mfma_i8(A[KMB - 1][s], ring[s & (NR - 1)], s == 0 ? seed[KMB - 1] : acc[p][1]);
      } else {
        acc[p][0] = mfma_i8(A[0][s], ring[s & (NR - 1)], s == 0 ? zero : acc[p][0]);
        if constexpr (KMB == 2) acc[p][1] = mfma_i8(A[KMB - 1][s], ring[s & (NR - 1)], s == 0 ? zero : acc[p][1]);
      }
      if constexpr (KMB == 2)
        asm volatile("" : "+v"(acc[p][0]), "+v"(acc[p][1]));
      else
        asm volatile("" : "+v"(acc[p][0]));
      if constexpr (s == FLS && !DENSE) {
        if (t >= 2) flush(t - 2, acc[p][0], acc[p][1]);
        VRQ_SCHED_FENCE();
      }
      // DMA of tile t + AHEAD, spread over the MFMA shadow
      if constexpr (P3) {
        if constexpr (s >= 2 && s < 2 + DS * PPW && (s - 2) % DS == 0)
          if (dma) issue_piece(dt, (s - 2) / DS);
      } else {
        if constexpr (s == 2)
          if (dma) issue_piece(dt, 0);
        if constexpr (s == 1) lds_read128(pv, sm0 + (uint32_t)(sl1 * T2) + usrc);
        if constexpr (s >= 5 && s < 5 + 2 * UD) unpack_frag(pv, s - 5, ubn);  // pv complete since step 3
      }
      // threshold test / dense value of tile t-1, one per k-step in [EOFF, EOFF + NE)
      constexpr int EOFF = KNE == 16 ? 4 : 0;
      if constexpr (s >= EOFF && s < EOFF + KNE) {
        constexpr int e = s - EOFF;
        if constexpr (!first) {
          if constexpr (SEED2)
            itest(acc[p ^ 1][0], acc[p ^ 1][1], e);
          else
            test(uval(acc[p ^ 1][0], acc[p ^ 1][1], e, invp), e, vprev);
          // pin the test's running state at this k-step: the tests are pure arithmetic, and without
          // a use here IR-level sinking gathers all of them after the tile's last MFMAs (past the
          // norm branch at s = 20), one ~90-instruction burst per tile instead of a few instructions
          // in each MFMA gap
          if constexpr (SEED2)
            asm volatile("" : "+v"(imax), "+v"(iodd));
          else if constexpr (DENSE)
            asm volatile("" : "+v"(ures[e]));
          else
            asm volatile("" : "+s"(hmk[e]));
        }
      }
      if constexpr (P3 && s == 20) {  // 1/||x|| of this tile's row r (NaN: zero norm or past the end)
        // (branch-free: a short-circuit && here splits the tile's basic block and its schedule)
        const float rc = __builtin_amdgcn_rcpf((float)nv);
        invc = ((nv > 0.0) & lane_valid(t)) ? rc : __builtin_nanf("");
      }
      VRQ_SCHED_FENCE();
    });
    invpp = invp;
    invp = invc;
    sl = sl1;
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using NOTFIRST = std::integral_constant<bool, false>;
  tile(I0{}, std::integral_constant<bool, true>{}, 0);
  int t = 1;
  for (; t + 1 < ntiles; t += 2) {
    tile(I1{}, NOTFIRST{}, t);
    tile(I0{}, NOTFIRST{}, t + 1);
  }
  if (t < ntiles) tile(I1{}, NOTFIRST{}, t);
  wait_vm<0>();
  // tile ntiles-2 (tested during the last tile), then the last tile itself
  const int pl = (ntiles - 1) & 1;
  if (!DENSE && ntiles >= 2) {
    if (pl)
      flush(ntiles - 2, acc[0][0], acc[0][1]);
    else
      flush(ntiles - 2, acc[1][0], acc[1][1]);
  }
  const bool vlast = lane_valid(ntiles - 1);
#pragma unroll
  for (int e = 0; e < KNE; ++e) {
    if constexpr (SEED2) {
      if (pl)
        itest(acc[1][0], acc[1][1], e);
      else
        itest(acc[0][0], acc[0][1], e);
    } else {
      test(pl ? uval(acc[1][0], acc[1][1], e, invp) : uval(acc[0][0], acc[0][1], e, invp), e, vlast);
    }
  }
  if constexpr (DENSE) {  // the lane maxima of the chunk -> dv[q][chunk * 32 + r]
#pragma unroll
    for (int e = 0; e < KNE; ++e) {
      const int q = qbase + qrow(e);
      if (q < nq) dv[(int64_t)q * dv_stride + (int64_t)chunk * GRT + r] = ures[e];
    }
  } else if (pl) {
    flush(ntiles - 1, acc[1][0], acc[1][1]);
  } else {
    flush(ntiles - 1, acc[0][0], acc[0][1]);
  }
  if constexpr (!DENSE) {
    drain();
    wait_lgkm0();
    if (l < KQW && qbase + l < nq) ccnt[(int64_t)(qbase + l) * nchunks + chunk] = lcnt[w * KQW + l];
  }
}

// ---------------------------------------------------------------------------------------------
// select: per query, U = k-th largest valid value of dv (the sample pass's lane maxima: nsc chunks of
// scr = 32 values; 3-pass radix select on the monotone key),
// thr = U - 2 Delta rounded down (-inf when the sample holds fewer than k finite values); zeroes the
// query's list lengths for the main pass.  Padding queries get thr = +inf.
__global__ __launch_bounds__(256) void gemm_select_kernel(const float* __restrict__ dv, int64_t dv_stride,
                                                          int64_t scr, int64_t sstride, int nsc, int64_t n, int k,
                                                          const double* __restrict__ delta, float* __restrict__ thr,
                                                          int32_t* __restrict__ ccnt, int nchunks, int nq,
                                                          int32_t* __restrict__ qbflag, int nqb) {
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t res[3];
  const int q = blockIdx.x, tid = threadIdx.x;
  if (q == 0)
    for (int i = tid; i < nqb; i += 256) qbflag[i] = 0;
  if (q >= nq) {
    if (tid == 0) thr[q] = __builtin_inff();
    return;
  }
  for (int i = tid; i < nchunks; i += 256) ccnt[(int64_t)q * nchunks + i] = 0;
  const float* d = dv + (int64_t)q * dv_stride;
  uint32_t prefix = 0, pmask = 0;
  int kk = k;
  bool ok = true;
  constexpr int SH[3] = {21, 10, 0}, NBITS[3] = {11, 11, 10};
  for (int pass = 0; pass < 3 && ok; ++pass) {
    const int sh = SH[pass];
    const uint32_t dm = (1u << NBITS[pass]) - 1;
    for (int i = tid; i < 2048; i += 256) hist[i] = 0;
    __syncthreads();
    for (int c = 0; c < nsc; ++c) {
      const int64_t rb = (int64_t)c * sstride;
      const int64_t len = (rb + scr <= n) ? scr : (n > rb ? n - rb : 0);
      const float* dc = d + (int64_t)c * scr;
      for (int64_t i = tid; i < len; i += 256) {
        const uint32_t key = fkey(dc[i]);
        if ((key & pmask) == prefix) atomicAdd(&hist[(key >> sh) & dm], 1u);
      }
    }
    __syncthreads();
    if (tid < 64) {  // top-down search: lane L owns bins [32L, 32L + 32)
      uint32_t loc = 0;
      for (int i = 0; i < 32; ++i) loc += hist[tid * 32 + i];
      uint32_t suf = loc;  // inclusive suffix sum over lanes >= tid
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_down(suf, o, 64);
        if (tid + o < 64) suf += y;
      }
      uint32_t above = suf - loc;
      int found = -1;
      uint32_t abv = 0;
      for (int i = 31; i >= 0; --i) {
        const uint32_t hc = hist[tid * 32 + i];
        if (above < (uint32_t)kk && above + hc >= (uint32_t)kk) {
          found = tid * 32 + i;
          abv = above;
        }
        above += hc;
      }
      const uint64_t bal = __ballot(found >= 0);
      if (tid == 0) res[0] = bal ? 1u : 0u;
      if (found >= 0) {
        res[1] = (uint32_t)found;
        res[2] = abv;
      }
    }
    __syncthreads();
    if (!res[0]) {
      ok = false;
    } else {
      const uint32_t b = res[1];
      kk -= (int)res[2];
      prefix |= b << sh;
      pmask |= dm << sh;
    }
    __syncthreads();
  }
  if (tid == 0) {
    float t = -__builtin_inff();
    if (ok && prefix != 0u) {
      const double U = (double)fkey_inv(prefix);
      t = __double2float_rd(U - 2.0 * delta[q]);
    }
    thr[q] = t;
  }
}

// ---------------------------------------------------------------------------------------------
// exact (score desc, row asc) pair sort in LDS: ascending (key, row), key = desc_key_f64(score)
__device__ inline void block_sort_pairs(uint64_t* key, uint32_t* row, int n_pow2) {
  for (int size = 2; size <= n_pow2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < (n_pow2 >> 1); i += blockDim.x) {
        const int lo = ((i / stride) * stride * 2) + (i % stride), hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t ka = key[lo], kb = key[hi];
        const uint32_t ra = row[lo], rb = row[hi];
        const bool gt = ka > kb || (ka == kb && ra > rb);
        if (gt == up) {
          key[lo] = kb;
          key[hi] = ka;
          row[lo] = rb;
          row[hi] = ra;
        }
      }
    }
  }
  __syncthreads();
}

// the corpus arrays a score reads (unused ones NULL)
struct Rows {
  const uint8_t* codes;  // VRQ_GEMM_BINARY: packed ubinary rows
  const int8_t* x8;      // VRQ_GEMM_INT8_COSINE: int8 rows
  const double* norms;   //   ... and their ||int8||_2
  const float* xf;       // VRQ_GEMM_FLOAT_IP: float32 rows
};

// The exact score of one row in two halves: the lane's load of the row (so a wave can keep several
// candidates' loads in flight) and the arithmetic (exact_scores.h, bit-identical to the fused search).
template <int PH>
struct RowSlice {
  int4 x;      // Phase III: the lane's 16 int8 values
  double nrm;  //   ... and the row's norm
};
template <>
struct RowSlice<VRQ_GEMM_BINARY> {
  uint16_t b;  // the lane's two code bytes
};
template <>
struct RowSlice<VRQ_GEMM_FLOAT_IP> {
  FlatSlice x;  // the lane's 16 floats
};
template <int PH>
__device__ __forceinline__ RowSlice<PH> load_row(const Rows& c, int64_t row) {
  RowSlice<PH> d;
  if constexpr (PH == VRQ_GEMM_BINARY) {
    d.b = phase2_load(c.codes + row * (DIM / 8));
  } else if constexpr (PH == VRQ_GEMM_FLOAT_IP) {
    d.x = flat_load(c.xf + row * DIM);
  } else {
    d.x = phase3_load(c.x8 + row * DIM);
    d.nrm = c.norms[row];
  }
  return d;
}
template <int PH>
__device__ __forceinline__ double score_row(const float (&qv)[DPL], const RowSlice<PH>& d) {
  if constexpr (PH == VRQ_GEMM_BINARY)
    return phase2_from(qv, d.b);
  else if constexpr (PH == VRQ_GEMM_FLOAT_IP)
    return flat_from(qv, d.x);
  else
    return phase3_from(qv, d.x, d.nrm);
}
// candidate rows a wave scores per round, all loads issued before the first score.  Measured at
// 10M rows (c5 finish, ms per 1024 queries; profiles/r2s3/c5_finish_score_batch.jsonl):
//   binary  1 row 0.89, 2 rows 0.78, 3 rows 0.75, 8 rows 1.25
//   cosine  1 row 1.23, 2 rows 1.13, 3 rows 1.15, 8 rows 1.79
// (more rows per round cost VGPRs and with them resident workgroups per CU).
// Round 6: those rounds had every load under `if (row < end)`, and a load under a divergent branch gets
// its own vmcnt(0) at the join, so the "batched" loads were issued one at a time; the loads are now
// unconditional (rows past the end re-read the last one).
#ifndef VRQ_SCORE_BATCH2
#define VRQ_SCORE_BATCH2 3
#endif
#ifndef VRQ_SCORE_BATCH3  // round 6, with the loads truly in flight together: 2 / 4 / 6 rows -> cosine
#define VRQ_SCORE_BATCH3 6  // finish 0.77-0.80 / 0.74-0.75 / 0.72-0.74 ms (profiles/r6_c5_cosine_batch_ab.jsonl)
#endif
template <int PH>
constexpr int kScoreBatch = PH == VRQ_GEMM_BINARY ? VRQ_SCORE_BATCH2 : VRQ_SCORE_BATCH3;

// Running exact top-k over a sequence of candidate rows row_at(j), j < count: every row is scored
// exactly (one wave per row); a row enters the LDS sort only if it beats the current k-th by
// (score desc, row asc), so the sort runs rarely once the list is full.  key/row[0..kc) hold the
// running list in order.  All threads of the block call it; returns kc = min(k, count).
// Binary (Phase II) with `qtab` (phase2_table of the query): one candidate row per THREAD, scored by the
// nibble table (256 LDS lookups; round 6) instead of one row per wave.
template <int PH, int NW = 4, class RowAt>
__device__ int running_topk(int64_t count, RowAt row_at, const float (&qv)[DPL], const Rows& c, int k,
                            uint64_t* key, uint32_t* row, int32_t* fill, uint32_t* bid = nullptr,
                            const double* qtab = nullptr) {
  constexpr int NT = NW * WAVE;
  const int tid = threadIdx.x, l = lane_id(), w = tid >> 6;
  if (tid == 0) *fill = 0;
  int kc = 0;
  __syncthreads();
  for (int64_t base = 0; base < count; base += FB_BATCH) {
    const uint64_t kk = kc == k ? key[k - 1] : KEY_NONE;
    const uint32_t kr = kc == k ? row[k - 1] : 0xffffffffu;
    const int64_t end = base + FB_BATCH < count ? base + FB_BATCH : count;
    constexpr int U = kScoreBatch<PH>;
    if (bid) {  // the batch's row ids -> LDS by all threads at once (row_at may read global memory)
      for (int64_t j = base + tid; j < end; j += NT) bid[j - base] = row_at(j);
      __syncthreads();
    }
    if constexpr (PH == VRQ_GEMM_BINARY) {
      if (qtab) {  // one candidate per thread
        for (int64_t j = base + tid; j < end; j += NT) {
          const uint32_t rr = bid ? bid[j - base] : row_at(j);
          const uint64_t key_r = desc_key_f64(phase2_nibbles(qtab, c.codes + (int64_t)rr * (DIM / 8)));
          if (kc < k || key_r < kk || (key_r == kk && rr < kr)) {
            const int i = kc + atomicAdd(fill, 1);
            key[i] = key_r;
            row[i] = rr;
          }
        }
      }
    }
    for (int64_t j0 = base + w; j0 < end && !(PH == VRQ_GEMM_BINARY && qtab); j0 += NW * U) {  // one row per wave
      uint32_t rr[U];
      RowSlice<PH> d[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t jj = j0 + NW * u < end ? j0 + NW * u : end - 1;  // (j0 < end)
        rr[u] = bid ? bid[jj - base] : row_at(jj);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) d[u] = load_row<PH>(c, (int64_t)rr[u]);  // unconditional: one wait for all
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (j0 + NW * u >= end) break;
        const uint64_t key_r = desc_key_f64(score_row<PH>(qv, d[u]));
        const bool take = kc < k || key_r < kk || (key_r == kk && rr[u] < kr);
        if (take && l == 0) {
          const int i = kc + atomicAdd(fill, 1);
          key[i] = key_r;
          row[i] = rr[u];
        }
      }
    }
    __syncthreads();
    const int f = *fill;
    if (f > 0) {
      const int tot = kc + f;
      const int np2 = next_pow2(tot);
      for (int i = tot + tid; i < np2; i += NT) {
        key[i] = KEY_NONE;
        row[i] = 0xffffffffu;
      }
      block_sort_pairs(key, row, np2);
      kc = tot < k ? tot : k;
    }
    if (tid == 0) *fill = 0;
    __syncthreads();
  }
  return kc;
}

constexpr int MAX_CHUNKS = 2048;  // per-query candidate lists the finish kernel indexes
// finish: threads per query (one workgroup each).  Measured at 10M rows, nq = 1024 (~1.8K Phase-III /
// ~1.3K Phase-II candidates per query, evenly spread: p99 / mean 1.2-1.4, tools/c5_candidates.py):
// 256 threads 0.86 / 0.51 ms, 512 threads 0.80 / 0.47 ms, 1024 threads 0.93 / 0.58 ms (Phase III /
// Phase II; profiles/r3_c5_finish_variants.jsonl).
constexpr int FIN_NT = 512, FIN_NW = FIN_NT / WAVE;
struct FinShared {
  uint64_t key[KMAX5 + FB_BATCH];
  uint32_t row[KMAX5 + FB_BATCH];
  uint32_t bid[FB_BATCH];       // the current batch's candidate rows
  int32_t pre[MAX_CHUNKS + 1];  // exclusive prefix of the list lengths
  int32_t misc[4];
};

// finish: the query's candidate lists -> exact scores -> running top-k -> first min(k, n), with the
// query's flag (fb_flag): 0 = served; 2 = retry; 1 = exact fallback.
//   A list overflow (more rows passed the sampled threshold than a list holds: a query whose
//   neighbourhood the sample under-represents) with >= min(k, n) recorded candidates -> RETRY: the
//   k-th best exact score s_k among the recorded candidates is a lower bound of the true k-th score,
//   so every row of the exact top-k (ties with the k-th included) has u >= alpha s_k + beta - Delta;
//   that raised threshold goes to thr[q] and the query block to the retry main pass.
//   Fewer than min(k, n) candidates (zero-norm rows) -> the fallback.
// Pass 2 (RETRY = true) serves the retried queries from the retry pass's lists; an overflow there
// goes to the fallback.  A served or abandoned query's thr becomes +inf, so a retry pass over its
// query block records nothing for it.
template <int PH, bool RETRY>
__global__ __launch_bounds__(FIN_NT, 4) void gemm_finish_kernel(const Rows c, int64_t n,  // (<= 128 VGPRs: 2 per CU)
                                                          int64_t row_offset, const float* __restrict__ qf, int k,
                                                          const uint32_t* __restrict__ cand,
                                                          const int32_t* __restrict__ ccnt, int nchunks, int capc,
                                                          int32_t* __restrict__ out_count,
                                                          int64_t* __restrict__ out_rows,
                                                          double* __restrict__ out_scores,
                                                          int32_t* __restrict__ fb_flag, float* __restrict__ thr,
                                                          const double* __restrict__ alpha,
                                                          const double* __restrict__ beta,
                                                          const double* __restrict__ delta,
                                                          int32_t* __restrict__ qbflag) {
  __shared__ FinShared sh;
  const int q = blockIdx.x, tid = threadIdx.x;
  if (RETRY && fb_flag[q] != 2) return;
  if (tid == 0) sh.misc[1] = 0;  // overflow
  __syncthreads();
  const int32_t* cq = ccnt + (int64_t)q * nchunks;
  // exclusive prefix of the (capped) list lengths: thread t owns chunks [t * per, t * per + per),
  // all its loads in flight at once, then a block scan of the FIN_NT partial sums (a serial loop over
  // the chunks cost one dependent global load per chunk)
  {
    constexpr int PER_MAX = (MAX_CHUNKS + FIN_NT - 1) / FIN_NT;
    const int per = (nchunks + FIN_NT - 1) / FIN_NT, c0 = tid * per;
    int v[PER_MAX];
    int part = 0;
#pragma unroll
    for (int i = 0; i < PER_MAX; ++i) {
      const int c = c0 + i;
      const int x = (i < per && c < nchunks) ? cq[c] : 0;
      if (x > capc) atomicOr(&sh.misc[1], 1);
      v[i] = x < capc ? x : capc;
      part += v[i];
    }
    // inclusive scan of `part` over the block: wave scan (shuffles), then the 4 wave totals
    int incl = part;
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
      const int y = __shfl_up(incl, d, WAVE);
      if (lane_id() >= d) incl += y;
    }
    __shared__ int wtot[FIN_NW];
    if (lane_id() == WAVE - 1) wtot[tid >> 6] = incl;
    __syncthreads();
    int off = 0;
    for (int ww = 0; ww < (tid >> 6); ++ww) off += wtot[ww];
    int acc = off + incl - part;  // exclusive prefix of this thread's first chunk
#pragma unroll
    for (int i = 0; i < PER_MAX; ++i) {
      const int c = c0 + i;
      if (i < per && c < nchunks) {
        sh.pre[c] = acc;
        acc += v[i];
      }
    }
    if (tid == FIN_NT - 1) sh.pre[nchunks] = off + incl;
  }
  __syncthreads();
  const int total = sh.pre[nchunks];
  const int need = (int)((int64_t)k < n ? k : n);
  if (total < need || (RETRY && sh.misc[1])) {
    if (tid == 0) {
      fb_flag[q] = 1;
      thr[q] = __builtin_inff();
    }
    return;
  }
  const uint32_t* Cq = cand + (int64_t)q * nchunks * capc;
  auto row_at = [&](int64_t j) {  // candidate j of the concatenated lists (binary search by chunk)
    int lo = 0, hi = nchunks - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sh.pre[mid] <= j)
        lo = mid;
      else
        hi = mid - 1;
    }
    return Cq[(int64_t)lo * capc + (j - sh.pre[lo])];
  };
  float qv[DPL];
  load_q(qv, qf + (int64_t)q * DIM);
  __shared__ double qtab[PH == VRQ_GEMM_BINARY ? 256 * 16 : 1];
  if constexpr (PH == VRQ_GEMM_BINARY) {
    phase2_table(qf + (int64_t)q * DIM, qtab, tid, FIN_NT);
    __syncthreads();
  }
  const int kc = running_topk<PH, FIN_NW>(total, row_at, qv, c, k, sh.key, sh.row, &sh.misc[2], sh.bid,
                                          PH == VRQ_GEMM_BINARY ? qtab : nullptr);
  if (!RETRY && sh.misc[1]) {  // overflow: raise the threshold to the recorded k-th score, retry
    if (tid == 0) {
      const double sk = desc_key_inv(sh.key[kc - 1]);
      const double t2 = alpha[q] * sk + beta[q] - delta[q];
      thr[q] = __double2float_rd(t2 - 1e-9 * fabs(t2));
      fb_flag[q] = 2;
      atomicOr(&qbflag[q / GQB], 1);
    }
    return;
  }
  for (int i = tid; i < k; i += FIN_NT) {
    const int64_t o = (int64_t)q * k + i;
    out_rows[o] = i < kc ? (int64_t)sh.row[i] + row_offset : -1;
    out_scores[o] = i < kc ? desc_key_inv(sh.key[i]) : __builtin_nan("");
  }
  if (tid == 0) {
    out_count[q] = kc;
    fb_flag[q] = 0;
    thr[q] = __builtin_inff();
  }
}

// fallback: exact running top-k over every row for the flagged queries (list overflow from heavy
// ties, zero-norm rows).  One workgroup per flagged query.
template <int PH>
__global__ __launch_bounds__(256) void gemm_fallback_kernel(const Rows c, int64_t n,
                                                            int64_t row_offset, const float* __restrict__ qf, int k,
                                                            int32_t* __restrict__ out_count,
                                                            int64_t* __restrict__ out_rows,
                                                            double* __restrict__ out_scores,
                                                            const int32_t* __restrict__ fb_flag,
                                                            bool skip) {
  __shared__ uint64_t key[KMAX5 + FB_BATCH];
  __shared__ uint32_t row[KMAX5 + FB_BATCH];
  __shared__ int32_t fill;
  const int q = blockIdx.x, tid = threadIdx.x;
  if (fb_flag[q] != 1) return;
  if (skip) {  // VRQ_GEMM_NO_FALLBACK: report the query as unserved
    for (int i = tid; i < k; i += 256) {
      out_rows[(int64_t)q * k + i] = -1;
      out_scores[(int64_t)q * k + i] = __builtin_nan("");
    }
    if (tid == 0) out_count[q] = -1;
    return;
  }
  float qv[DPL];
  load_q(qv, qf + (int64_t)q * DIM);
  __shared__ double qtab[PH == VRQ_GEMM_BINARY ? 256 * 16 : 1];
  if constexpr (PH == VRQ_GEMM_BINARY) {
    phase2_table(qf + (int64_t)q * DIM, qtab, tid, 256);
    __syncthreads();
  }
  const int kc = running_topk<PH>(n, [](int64_t j) { return (uint32_t)j; }, qv, c, k, key, row, &fill, nullptr,
                                  PH == VRQ_GEMM_BINARY ? qtab : nullptr);
  for (int i = tid; i < k; i += 256) {
    const int64_t o = (int64_t)q * k + i;
    out_rows[o] = i < kc ? (int64_t)row[i] + row_offset : -1;
    out_scores[o] = i < kc ? desc_key_inv(key[i]) : __builtin_nan("");
  }
  if (tid == 0) out_count[q] = kc;
}

// ---------------------------------------------------------------------------------------------
struct GemmPlan {
  int nqb, nq_pad;
  int64_t scr, sstride, scols;  // sample: nsc chunks of scr rows, chunk c at row c * sstride
  int nsc;
  int64_t chunk_rows;
  int nchunks, capc;
  size_t off_delta, off_alpha, off_beta, off_qbf, off_thr, off_flag, off_cnt, off_cand, off_dv, bytes;
};

static int gemm_plan(int64_t n, int nq, int k, GemmPlan* p) {
  if (n < 1 || n >= (int64_t(1) << 32) || nq < 1 || k < 1 || k > KMAX5) return VRQ_EUNSUPPORTED;
  p->nqb = (nq + GQB - 1) / GQB;
  p->nq_pad = p->nqb * GQB;
  // chunks per query block: kChunkMult per CU (VRQ_GEMM_CHUNK_MULT in the probe build): shorter
  // chunks keep the query blocks that share a chunk closer in time, so they share its L2 lines
  const int cm = tuning_int("VRQ_GEMM_CHUNK_MULT", kChunkMult);
  const int mult = cm >= 1 ? cm : kChunkMult;
  const int want1 = 256 / p->nqb > 0 ? 256 / p->nqb : 1;  // one workgroup per CU and query block
  const int want = want1 * mult;
  // sample rows: the sampled threshold alone admits ~k * n / S rows per query; aim at FIN_CAP /
  // CAP_MULT so that the margin's extra rows still fit (VRQ_GEMM_SAMPLE_DIV overrides n / S)
  int64_t S = (int64_t)((double)CAP_MULT * (double)k * (double)n / (double)FIN_CAP);
  const int ev = tuning_int("VRQ_GEMM_SAMPLE_DIV", 0);
  if (ev >= 1) S = n / ev;
  if (S < kMinSample) S = kMinSample;
  if (S > kMaxSample) S = kMaxSample;
  if (S > n) S = n;
  // sample chunks: one per CU and query block, and >= 2k / 32 so the select sees >= 2k lane maxima
  // per query (fewer than k would leave thr = -inf: every row a candidate)
  int64_t nsc = want1 > (2 * (int64_t)k + GRT - 1) / GRT ? want1 : (2 * (int64_t)k + GRT - 1) / GRT;
  int64_t scr = ((S + nsc - 1) / nsc + GRT - 1) / GRT * GRT;
  nsc = (S + scr - 1) / scr;
  p->scr = scr;
  p->nsc = (int)nsc;
  p->sstride = n / nsc >= scr ? n / nsc : scr;  // chunks never overlap; the last may be cut at n
  p->scols = nsc * GRT;  // dv columns per query: one running max per (sample chunk, lane row)
  int64_t cr = (n + want - 1) / want;
  cr = (cr + GRT - 1) / GRT * GRT;
  if ((n + cr - 1) / cr > MAX_CHUNKS) cr = ((n + MAX_CHUNKS - 1) / MAX_CHUNKS + GRT - 1) / GRT * GRT;
  // the thresholded pass's hit stage packs (query-in-wave << 26 | chunk row): chunks stay below 2^26
  // rows (n < 2^32 then needs at most 65 chunks, far below MAX_CHUNKS)
  if (cr > kMaxChunkRows) cr = kMaxChunkRows;
  p->chunk_rows = cr;
  p->nchunks = (int)((n + cr - 1) / cr);
  const int64_t Sv = S < n ? S : n;
  const int64_t expect = ((int64_t)k * cr + Sv - 1) / Sv;
  int capc = 64;
  while (capc < CAP_MULT * expect && capc < 4096) capc <<= 1;
  // headroom for neighbourhoods stored contiguously (a cluster in one chunk): at least 512 entries
  // per list while all lists of the batch stay within 1 GiB
  while (capc < 512 && (double)nq * p->nchunks * (2 * capc) * sizeof(uint32_t) <= (double)(1 << 30)) capc <<= 1;
  p->capc = capc;
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  const size_t qa = al((size_t)p->nq_pad * QA_BYTES);
  p->off_delta = qa;
  p->off_alpha = p->off_delta + al((size_t)p->nq_pad * sizeof(double));
  p->off_beta = p->off_alpha + al((size_t)p->nq_pad * sizeof(double));
  p->off_qbf = p->off_beta + al((size_t)p->nq_pad * sizeof(double));
  p->off_thr = p->off_qbf + al((size_t)p->nqb * sizeof(int32_t));
  p->off_flag = p->off_thr + al((size_t)p->nq_pad * sizeof(float));
  p->off_cnt = p->off_flag + al((size_t)nq * sizeof(int32_t));
  p->off_cand = p->off_cnt + al((size_t)nq * p->nchunks * sizeof(int32_t));
  p->off_dv = p->off_cand + al((size_t)nq * p->nchunks * p->capc * sizeof(uint32_t));
  p->bytes = p->off_dv + al((size_t)nq * p->scols * sizeof(float));
  return VRQ_OK;
}

// ---------------------------------------------------------------------------------------------
// IndexFlatIP corpus preparation (vrq_flat_ip_prepare): one wave per float32 row x_r.
//   s_r = max|x_r| / 127, b_r = clamp(rint(x_r / s_r), +-127) -> x8 (the matrix pass's int8 rows),
//   inv_scale[r] = 1 / s_r (the pass multiplies the exact i32 dot by fl32(1 / fl32(inv_scale)) =
//   s_r within 2^-22, inside the prep kernel's slack), and the running corpus bounds
//   bounds[0] = max ||s_r b_r||_2, bounds[1] = max ||x_r - s_r b_r||_2 (rounded up; atomic max of
//   the non-negative f64 bit patterns, so batches of adds accumulate).  Rows with max|x| < 1e-30
//   are stored as b = 0 (scale 1): the whole row is residual.
__global__ __launch_bounds__(256) void flat_ip_prepare_kernel(const float* __restrict__ xf, int64_t n,
                                                              int8_t* __restrict__ x8,
                                                              double* __restrict__ inv_scale,
                                                              unsigned long long* __restrict__ bounds) {
  __shared__ double sb[2][4];
  const int w = threadIdx.x >> 6, l = lane_id();
  const int64_t r = (int64_t)blockIdx.x * 4 + w;
  double ex = 0.0, es = 0.0;
  if (r < n) {
    float xv[DPL];
    load_q(xv, xf + r * DIM);
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < DPL; ++i) mx = fmaxf(mx, fabsf(xv[i]));
#pragma unroll
    for (int m = 1; m < WAVE; m <<= 1) mx = fmaxf(mx, __shfl_xor(mx, m, WAVE));
    const bool live = mx >= 1e-30f;
    const double sc = live ? (double)mx / 127.0 : 0.0, inv = live ? 127.0 / (double)mx : 0.0;
    double b2 = 0.0, s2 = 0.0;
    uint32_t pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < DPL; ++i) {
      double b = rint((double)xv[i] * inv);
      b = b > 127.0 ? 127.0 : (b < -127.0 ? -127.0 : b);
      const double rs = (double)xv[i] - sc * b;
      b2 += b * b;
      s2 += rs * rs;
      pk[i >> 2] |= ((uint32_t)(int32_t)b & 0xffu) << (8 * (i & 3));
    }
    *reinterpret_cast<int4*>(x8 + r * DIM + DPL * l) = make_int4((int)pk[0], (int)pk[1], (int)pk[2], (int)pk[3]);
    b2 = wave_sum_f64(b2);  // exact (integers < 2^24)
    s2 = wave_sum_f64(s2);
    ex = sc * sqrt(b2) * (1.0 + 1e-12);
    es = sqrt(s2) * (1.0 + 1e-12) + 1e-300;
    if (l == 0) inv_scale[r] = live ? inv : 1.0;
  }
  if (l == 0) {
    sb[0][w] = ex;
    sb[1][w] = es;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const double* v = sb[threadIdx.x];
    const double m = fmax(fmax(v[0], v[1]), fmax(v[2], v[3]));
    atomicMax(bounds + threadIdx.x, (unsigned long long)__double_as_longlong(m));
  }
}

}  // namespace g5
}  // namespace vrq

using namespace vrq;
using namespace vrq::g5;

extern "C" int vrq_gemm_topk_pieces(void) { return 1; }

namespace {

bool gemm_mode_ok(int mode) {
  return mode == VRQ_GEMM_BINARY || mode == VRQ_GEMM_INT8_COSINE || mode == VRQ_GEMM_FLOAT_IP;
}

// finish -> retry main pass (query blocks with a retried query) -> finish of the retried queries ->
// exact fallback of the rest
template <int PH>
void launch_finish(const Rows& c, const uint8_t* src, int64_t n, int64_t row_offset, const float* qf, int nq, int k,
                   const GemmPlan& p, const int8_t* qa, float* thr, uint32_t* cand, int32_t* cnt, int32_t* out_count,
                   int64_t* out_rows, double* out_scores, int32_t* flag, const double* alpha, const double* beta,
                   const double* delta, int32_t* qbf, bool fb, hipStream_t s) {
  constexpr int MP = PH == VRQ_GEMM_BINARY ? VRQ_GEMM_BINARY : VRQ_GEMM_INT8_COSINE;  // matrix-pass kind
  hipLaunchKernelGGL((gemm_finish_kernel<PH, false>), dim3(nq), dim3(FIN_NT), 0, s, c, n, row_offset, qf, k,
                     (const uint32_t*)cand, (const int32_t*)cnt, p.nchunks, p.capc, out_count, out_rows, out_scores,
                     flag, thr, alpha, beta, delta, qbf);
  hipLaunchKernelGGL((gemm_topk_kernel<MP, false, true>), dim3(p.nchunks * p.nqb), dim3(KShape<MP>::W * 64), 0, s, src, c.norms, n, qa,
                     nq, (const float*)thr, cand, cnt, p.capc, p.chunk_rows, p.chunk_rows, p.nchunks, p.nqb,
                     (float*)nullptr, (int64_t)0, (const int32_t*)qbf);
  hipLaunchKernelGGL((gemm_finish_kernel<PH, true>), dim3(nq), dim3(FIN_NT), 0, s, c, n, row_offset, qf, k,
                     (const uint32_t*)cand, (const int32_t*)cnt, p.nchunks, p.capc, out_count, out_rows, out_scores,
                     flag, thr, alpha, beta, delta, qbf);
  hipLaunchKernelGGL(gemm_fallback_kernel<PH>, dim3(nq), dim3(256), 0, s, c, n, row_offset, qf, k, out_count,
                     out_rows, out_scores, (const int32_t*)flag, !fb);
}

// The three stages shared by every mode.  The matrix passes of VRQ_GEMM_FLOAT_IP are the int8
// cosine passes over (the prepared int8 rows, 1/scale as the "norm"); only the prep kernel's bound
// and the exact score differ.
int gemm_run(int mode, const Rows& c, const double* bounds, int64_t n, int64_t row_offset, const float* qf, int nq,
             int k, int flags, int32_t* out_count, int64_t* out_rows, double* out_scores, void* workspace,
             size_t workspace_bytes, hipStream_t s) {
  GemmPlan p;
  const int rc = gemm_plan(n, nq, k, &p);
  if (rc != VRQ_OK) return rc;
  if (workspace_bytes < p.bytes) return VRQ_EWORKSPACE;
  constexpr int ALL = VRQ_GEMM_STAGE_SAMPLE | VRQ_GEMM_STAGE_MAIN | VRQ_GEMM_STAGE_FINISH;
  const int st = (flags & ALL) ? (flags & ALL) : ALL;
  uint8_t* ws = (uint8_t*)workspace;
  int8_t* qa = (int8_t*)ws;
  double* delta = (double*)(ws + p.off_delta);
  double* alpha = (double*)(ws + p.off_alpha);
  double* beta = (double*)(ws + p.off_beta);
  int32_t* qbf = (int32_t*)(ws + p.off_qbf);
  float* thr = (float*)(ws + p.off_thr);
  int32_t* flag = (int32_t*)(ws + p.off_flag);
  int32_t* cnt = (int32_t*)(ws + p.off_cnt);
  uint32_t* cand = (uint32_t*)(ws + p.off_cand);
  float* dv = (float*)(ws + p.off_dv);
  const bool P3 = mode != VRQ_GEMM_BINARY;  // int8 rows on the matrix cores
  const uint8_t* src = P3 ? (const uint8_t*)c.x8 : c.codes;
  const double* rn = c.norms;
  const dim3 blk(P3 ? KShape<VRQ_GEMM_INT8_COSINE>::W * 64 : KShape<VRQ_GEMM_BINARY>::W * 64);
  if (st & VRQ_GEMM_STAGE_SAMPLE) {
    hipLaunchKernelGGL(gemm_prep_kernel, dim3((p.nq_pad + 3) / 4), dim3(256), 0, s, mode, qf, nq, p.nq_pad, qa,
                       delta, alpha, beta, bounds);
    VRQ_LAUNCH_CHECK();
    const dim3 grid(p.nsc * p.nqb);
    if (P3)
      hipLaunchKernelGGL((gemm_topk_kernel<VRQ_GEMM_INT8_COSINE, true>), grid, blk, 0, s, src, rn, n, qa, nq,
                         (const float*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr, 0, p.scr, p.sstride, p.nsc,
                         p.nqb, dv, p.scols, (const int32_t*)nullptr);
    else
      hipLaunchKernelGGL((gemm_topk_kernel<VRQ_GEMM_BINARY, true>), grid, blk, 0, s, src, rn, n, qa, nq,
                         (const float*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr, 0, p.scr, p.sstride, p.nsc,
                         p.nqb, dv, p.scols, (const int32_t*)nullptr);
    VRQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(gemm_select_kernel, dim3(p.nq_pad), dim3(256), 0, s, (const float*)dv, p.scols, (int64_t)GRT,
                       p.sstride, p.nsc, n, k, (const double*)delta, thr, cnt, p.nchunks, nq, qbf, p.nqb);
    VRQ_LAUNCH_CHECK();
  }
  if (st & VRQ_GEMM_STAGE_MAIN) {
    const dim3 grid(p.nchunks * p.nqb);
    if (P3)
      hipLaunchKernelGGL((gemm_topk_kernel<VRQ_GEMM_INT8_COSINE, false>), grid, blk, 0, s, src, rn, n, qa, nq,
                         (const float*)thr, cand, cnt, p.capc, p.chunk_rows, p.chunk_rows, p.nchunks, p.nqb,
                         (float*)nullptr, (int64_t)0, (const int32_t*)nullptr);
    else
      hipLaunchKernelGGL((gemm_topk_kernel<VRQ_GEMM_BINARY, false>), grid, blk, 0, s, src, rn, n, qa, nq,
                         (const float*)thr, cand, cnt, p.capc, p.chunk_rows, p.chunk_rows, p.nchunks, p.nqb,
                         (float*)nullptr, (int64_t)0, (const int32_t*)nullptr);
    VRQ_LAUNCH_CHECK();
  }
  if (st & VRQ_GEMM_STAGE_FINISH) {
    // VRQ_GEMM_NO_FALLBACK: the flagged queries get out_count = -1 instead of the exact scan
    const bool fb = !(flags & VRQ_GEMM_NO_FALLBACK);
    const int8_t* qac = qa;
    const double *al = alpha, *be = beta, *de = delta;
    if (mode == VRQ_GEMM_INT8_COSINE)
      launch_finish<VRQ_GEMM_INT8_COSINE>(c, src, n, row_offset, qf, nq, k, p, qac, thr, cand, cnt, out_count,
                                          out_rows, out_scores, flag, al, be, de, qbf, fb, s);
    else if (mode == VRQ_GEMM_FLOAT_IP)
      launch_finish<VRQ_GEMM_FLOAT_IP>(c, src, n, row_offset, qf, nq, k, p, qac, thr, cand, cnt, out_count, out_rows,
                                       out_scores, flag, al, be, de, qbf, fb, s);
    else
      launch_finish<VRQ_GEMM_BINARY>(c, src, n, row_offset, qf, nq, k, p, qac, thr, cand, cnt, out_count, out_rows,
                                     out_scores, flag, al, be, de, qbf, fb, s);
    VRQ_LAUNCH_CHECK();
  }
  return VRQ_OK;
}

}  // namespace

extern "C" size_t vrq_gemm_topk_workspace_size(int32_t mode, int64_t n, int32_t dim, int32_t nq, int32_t k) {
  GemmPlan p;
  if (!gemm_mode_ok(mode) || dim != DIM || gemm_plan(n, nq, k, &p) != VRQ_OK) return 0;
  return p.bytes;
}

extern "C" int vrq_gemm_topk_plan(int32_t mode, int64_t n, int32_t dim, int32_t nq, int32_t k, int64_t* info) {
  GemmPlan p;
  if (!info) return VRQ_EINVAL;
  if (!gemm_mode_ok(mode) || dim != DIM) return VRQ_EUNSUPPORTED;
  const int rc = gemm_plan(n, nq, k, &p);
  if (rc != VRQ_OK) return rc;
  info[0] = p.chunk_rows;
  info[1] = p.nchunks;
  info[2] = p.capc;
  info[3] = p.nqb;
  info[4] = p.nsc;
  info[5] = p.scr;
  info[6] = (int64_t)p.bytes;
  info[7] = GQB;
  return VRQ_OK;
}

extern "C" int vrq_gemm_topk_layout(int32_t mode, int64_t n, int32_t dim, int32_t nq, int32_t k, int64_t* info) {
  GemmPlan p;
  if (!info) return VRQ_EINVAL;
  if (!gemm_mode_ok(mode) || dim != DIM) return VRQ_EUNSUPPORTED;
  const int rc = gemm_plan(n, nq, k, &p);
  if (rc != VRQ_OK) return rc;
  info[0] = p.nq_pad;
  info[1] = (int64_t)p.off_thr;
  info[2] = (int64_t)p.off_cnt;
  info[3] = (int64_t)p.off_cand;
  info[4] = (int64_t)p.off_dv;
  info[5] = p.scols;
  info[6] = p.sstride;
  info[7] = p.scr;
  return VRQ_OK;
}

extern "C" int vrq_gemm_topk(int32_t mode, const uint8_t* codes, const int8_t* x8, const double* norms, int64_t n,
                             int32_t dim, int64_t row_offset, const float* qf, int32_t nq, int32_t k, int32_t flags,
                             int32_t* out_count, int64_t* out_rows, double* out_scores, void* workspace,
                             size_t workspace_bytes, void* stream) {
  if (mode != VRQ_GEMM_BINARY && mode != VRQ_GEMM_INT8_COSINE) return VRQ_EINVAL;
  if (dim != DIM) return VRQ_EUNSUPPORTED;
  VRQ_CHECK_ARG(qf && out_count && out_rows && out_scores && workspace && n > 0 && nq > 0 && k > 0);
  if (mode == VRQ_GEMM_BINARY) VRQ_CHECK_ARG(codes);
  if (mode == VRQ_GEMM_INT8_COSINE) VRQ_CHECK_ARG(x8 && norms);
  const Rows c{codes, x8, norms, nullptr};
  return gemm_run(mode, c, nullptr, n, row_offset, qf, nq, k, flags, out_count, out_rows, out_scores, workspace,
                  workspace_bytes, (hipStream_t)stream);
}

extern "C" int vrq_flat_ip_prepare(const float* xf, int64_t n, int32_t dim, int8_t* x8, double* inv_scale,
                                   double* bounds, void* stream) {
  if (dim != DIM) return VRQ_EUNSUPPORTED;
  VRQ_CHECK_ARG(n >= 0 && bounds);
  if (n == 0) return VRQ_OK;
  VRQ_CHECK_ARG(xf && x8 && inv_scale);
  hipLaunchKernelGGL(flat_ip_prepare_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, xf, n,
                     x8, inv_scale, reinterpret_cast<unsigned long long*>(bounds));
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

extern "C" int vrq_flat_ip_topk(const float* xf, const int8_t* x8, const double* inv_scale, const double* bounds,
                                int64_t n, int32_t dim, int64_t row_offset, const float* qf, int32_t nq, int32_t k,
                                int32_t flags, int32_t* out_count, int64_t* out_rows, double* out_scores,
                                void* workspace, size_t workspace_bytes, void* stream) {
  if (dim != DIM) return VRQ_EUNSUPPORTED;
  VRQ_CHECK_ARG(xf && x8 && inv_scale && bounds && qf && out_count && out_rows && out_scores && workspace && n > 0 &&
                nq > 0 && k > 0);
  const Rows c{nullptr, x8, inv_scale, xf};
  return gemm_run(VRQ_GEMM_FLOAT_IP, c, bounds, n, row_offset, qf, nq, k, flags, out_count, out_rows, out_scores,
                  workspace, workspace_bytes, (hipStream_t)stream);
}
