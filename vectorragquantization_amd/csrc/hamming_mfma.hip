// hamming_mfma.hip -- K1m: Phase-I Hamming scan for LARGE query batches on the matrix cores.
//
// The wavefront popcount scan (hamming_scan.hip) costs 64 wave64 VALU instructions per
// (query, 1024-bit row) pair and a wave64 integer VALU op retires every 4 cycles
// (tools/probes/valu_probe.hip): beyond ~16 queries per pass it is VALU-bound.  Here the
// same distances come from the block-scaled FP4 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4) on
// 0/1 e2m1 values:
//     dist(q, r) = popcount(q) + popcount(r) - 2 * <bits(q), bits(r)>
// which is exact (integer values in f32), so Phase-I ranks stay bit-identical to FAISS.
//
// Work decomposition: one 256-thread workgroup per CU (LDS ~138 KiB), one wave per SIMD:
//  * each wave holds the A fragments of 64 queries (2 M-blocks of 32) for the whole K = 1024
//    in the accumulator register file (128 AGPRs, unpacked once) and their thresholds folded
//    into the accumulator seeds; accumulators, seeds and the B ring live in VGPRs, so the
//    epilogue reads results where the MFMA wrote them;
//  * 64-row tiles of PACKED codes stream HBM -> LDS by LDS-DMA (XOR-swizzled source, ring of
//    4); while the matrix core runs tile t, the same waves expand tile t+2 into FP4 B
//    fragments laid out [n-block][k-step][lane][16 B] (one contiguous ds_read_b128 per
//    fragment) plus the rows' popcounts -- VALU work in the gaps between MFMAs.  One barrier
//    per tile publishes the unpacked tile (ring of 3);
//  * each B fragment feeds the MFMAs of BOTH M-blocks (LDS reads: 32 KiB per wave per tile);
//  * epilogue per n-block, in the next n-block's MFMA shadow: a row is a candidate iff
//    dist < tau(q), tau(q) = the exact K-th smallest distance of the query over a PREFIX of
//    the corpus (computed by the exact scan).  FAISS admits a row only if dist < heap_top,
//    rows in increasing index: a suffix row with dist >= tau(q) ranks after >= K prefix rows,
//    so the strict test loses nothing.  A max3 tree + one compare per (M-block, lane) rejects
//    hit-free blocks; hits are ballot-compacted into a per-wave LDS stage of packed 32-bit
//    entries and, once per tile, appended to per-(query, chunk) lists in HBM at positions
//    taken from per-query LDS counters.  suffix_topk_kernel merges the lists into one sorted
//    K-list per query, exactly in every case (overflow -> exact rescan).
#include <stdlib.h>

#include "mfma_common.h"
#include "vrq_internal.h"
#include "vrq_scan.h"

namespace vrq {

constexpr int MWAVES = 4;                   // waves per workgroup (one per SIMD)
constexpr int RT = 64;                      // rows per tile (2 n-blocks of 32)
constexpr int KS = 16;                      // k-steps of 64 bits (1024-bit codes)
constexpr int NG = 2 * KS;                  // k-step groups per tile (n-block, k-step)
constexpr int PKT = RT * 128;               // packed tile bytes (8 KiB)
constexpr int NPK = 4;                      // packed ring depth (DMA issued NPK tiles ahead)
constexpr int NUB = 3;                      // unpacked ring: tile t read, t+1 ready, t+2 written
constexpr int UBT = NG * 1024;              // unpacked tile bytes (32 KiB)
constexpr int GPW = (PKT / 1024) / MWAVES;  // LDS-DMA instructions per wave per tile (2)
constexpr int BAHEAD = 3;                   // B fragments read this many groups ahead
constexpr int NRING = BAHEAD < 4 ? 4 : 8;   // B fragment ring (power of two > BAHEAD)
constexpr int STG = 512;                    // per-wave staged hit entries (u32)
constexpr int FMT_FP4 = 4;                  // e2m1 operand format of the f8f6f4 MFMA
#ifndef VRQ_K1M_DMA_AHEAD  // A/B builds: K1m refills a packed slot one iteration earlier (two tiles of DMA lead)
#define VRQ_K1M_DMA_AHEAD 0
#endif
// M-blocks (32 queries each) per wave: MB = 4 for large batches (512 queries per workgroup, each
// B fragment feeds 4 MFMAs), MB = 2 below (256 per workgroup)
template <int MB>
struct MfmaShape {
  static constexpr int QPW = 32 * MB;                 // queries per wave
  static constexpr int QPB = MWAVES * QPW;            // queries per workgroup
  static constexpr int SMEM =
      NPK * PKT + NUB * UBT + NUB * RT * 4 + MWAVES * QPW * 8 + MWAVES * (STG + 1) * 4 + MWAVES * MB * 128;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
};
constexpr int kMbLarge = 4, kMbSmall = 2;
constexpr int kMbLargeMinQueries = 512;     // batches of >= 512 queries take the MB = 4 kernel
constexpr int kRowsMaxQueries = 128;        // batches of <= 128 queries take the row-split kernel K1r

// 32 code bits -> one FP4 MFMA fragment lane: 32 e2m1 values.  Dword j, nibble i holds bit 4i + j
// (a fixed permutation of k applied identically to queries and rows, so every dot product is
// unchanged), encoded so that A x B = 1 per common set bit:
//   rows (B):    j = 0, 1, 2: w & (0x11111111 << j) -> codes 0x1 / 0x2 / 0x4 = 0.5 / 1 / 2;
//                j = 3: (w >> 1) & 0x44444444 -> 0x4 = 2           (5 VALU per 32 bits)
//   queries (A): 2 / 1 / 0.5 / 0.5 at the same positions (unpacked once per kernel)
__device__ __forceinline__ v4i unpack_row32(uint32_t w) {
  v4i r;
  r.x = (int)(w & 0x11111111u);
  r.y = (int)(w & 0x22222222u);
  r.z = (int)(w & 0x44444444u);
  r.w = (int)((w >> 1) & 0x44444444u);
  return r;
}
__device__ __forceinline__ v4i unpack_query32(uint32_t w) {
  v4i r;
  r.x = (int)((w << 2) & 0x44444444u);
  r.y = (int)(w & 0x22222222u);
  r.z = (int)((w >> 2) & 0x11111111u);
  r.w = (int)((w >> 3) & 0x11111111u);
  return r;
}

// Unscaled v_mfma_f32_32x32x64_f8f6f4 (scale operands 0 select the unscaled form, 32 cycles; the
// block-scaled form costs 33 on these operands, tools/probes/mfma_shape_probe.hip): 1 per common
// set bit (unpack_row32 x unpack_query32), so C + popcount(q & r) exactly (integers <= 1024 in f32).
// FP4 operands occupy 4 registers; the upper half of the 8-register operand is ignored.
__device__ __forceinline__ v16f mfma_fp4(const v4i& a, const v4i& b, const v16f& c) {
  const v8i a8 = {a.x, a.y, a.z, a.w, 0, 0, 0, 0};
  const v8i b8 = {b.x, b.y, b.z, b.w, 0, 0, 0, 0};
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, c, FMT_FP4, FMT_FP4, 0, 0, 0, 0);
}


// Packed tile image: 16-byte piece c of tile row r lives at slot r*8 + (c ^ ((r>>1)&7)).
__device__ __forceinline__ int pk_slot(int r, int c) { return r * 8 + (c ^ ((r >> 1) & 7)); }

// wave-uniform "any lane has a value > thr in these 16 registers", for thr >= 0: a signed-integer
// max3 tree over the float bit patterns (non-negative floats order like their bits; negative ones
// are below every non-negative pattern, and none of them can exceed thr >= 0), no canonicalisation
__device__ __forceinline__ bool any_above(const v16f& a, float thr) {
  const v16i b = __builtin_bit_cast(v16i, a);
  // tree of depth 3: five independent max3, then two, then one
  const int x0 = max(max(b[0], b[1]), b[2]), x1 = max(max(b[3], b[4]), b[5]), x2 = max(max(b[6], b[7]), b[8]);
  const int x3 = max(max(b[9], b[10]), b[11]), x4 = max(max(b[12], b[13]), b[14]);
  const int y0 = max(max(x0, x1), x2), y1 = max(max(x3, x4), b[15]);
  return __ballot(max(y0, y1) > __float_as_int(thr)) != 0;
}

// Staged hit entry (u32): (v + 1025) << 14 | query-in-wave << 7 | row - (t-1)*64, where
// v = dist - tau(q) in [-1025, -1] (tau = the threshold the pass ran with; the suffix kernel adds it
// back) and the row is relative to the previous tile's first row (the epilogue of a tile's second
// n-block runs in the next tile's iteration).  List keys carry the same field: (v + 1025) << 40 | row.
constexpr int ENT_V_SHIFT = 14, ENT_Q_SHIFT = 7, ENT_V_BIAS = 1025;

// DENSE = the sample pass: no thresholds; every (query, row) pair's v = dist - pc(q) folds into
// the lane's running minima (dense_out below), written once per chunk.  Chunk c
// starts at row row_begin + c * chunk_stride and its tile t at + t * tile_stride: the sample pass
// spreads 64-row tiles evenly over the whole corpus (tile_stride >= 64, chunk_rows = its tiles x 64
// dv columns); the thresholded pass uses chunk_stride = chunk_rows and tile_stride = 64.
// MODE: MFMA_MAIN (thresholded pass), MFMA_SAMPLE (dense sample pass, DENSE below) or MFMA_RERUN
// (the exact re-run of failed query blocks: same code as MAIN, a separate symbol so profiles and
// traces tell the two launches apart).
//
// Schedule of the 32 k-step groups of a tile (group gi = (n-block gi>>4, k-step j = gi&15)): every
// group reads the B fragment of group gi+BAHEAD (one ds_read_b128, immediate offset) and runs MB
// MFMAs on the fragment of group gi.  Around them, spread so no group's vector work much exceeds
// its MFMA shadow: the packed reads of unpack unit u (gi = 8u+1) and its unpack + LDS writes
// (gi = 8u+6), the row-popcount reads (gi = 12) and writes (gi = 28); for the previous n-block the
// hit test of M-block m (j = 2+m), one branch to the (rare) hit extraction (j = 3+MB) and the
// accumulator re-seeds (j = 4+MB, two M-blocks per group); the asynchronous hit flush
// (gi = 20+MB and 24+MB).
enum { MFMA_MAIN = 0, MFMA_SAMPLE = 1, MFMA_RERUN = 2 };

// The per-group LDS wait of the schedule above.  Group gi consumes the B fragment read at the top of
// group gi - BAHEAD; DS operations complete in order, so the wait may leave in flight exactly the DS
// operations issued after that read: the B reads of the groups since, and every other LDS operation
// of those groups on the no-hit path (a hit adds stage writes, which only makes the counted wait
// stricter).  Per group g: pre(g) = reads issued after its B read and before its wait (packed unit,
// row popcounts), post(g) = operations issued in its slots (unpack writes, the popcount write, four
// accumulator-seed reads, the two hit-flush steps).  Groups gi < BAHEAD read tiles the previous
// iteration's lgkmcnt(0) retired: their wait counts this iteration's operations so far.  Capped at 15
// (the counter's range; a smaller count only waits longer).
constexpr int k1m_pre(int g) { return ((g & 7) == 1 ? 1 : 0) + (g == 12 ? 2 : 0); }
constexpr int k1m_post(int g, int mb, bool dense) {
  const int j = g & 15;
  return ((g & 7) == 6 ? 2 : 0) + (g == 28 ? 1 : 0) + (!dense && j >= 4 + mb && j < 4 + 2 * mb ? 4 : 0) +
         (!dense && g == 20 + mb ? 1 : 0) + (!dense && g == 24 + mb ? 1 : 0);
}
constexpr int k1m_wait(int gi, int mb, bool dense) {
  const int g0 = gi - BAHEAD;
  int n = 1 + k1m_pre(gi);  // this group's B read and pre-wait reads
  for (int g = g0 < 0 ? 0 : g0; g < gi; ++g) n += (g == g0 ? 0 : 1) + k1m_pre(g) + k1m_post(g, mb, dense);
  return n < 15 ? n : 15;
}

// The dense sample pass keeps, per lane and accumulator register, the minimum of v = dist - pc(q)
// over the sample rows of its chunk that the lane holds (lane row ri of every n-block): 32 values
// per (query, chunk), each the distance of a DISTINCT sample row, written once per chunk as u16
// (v + 1024; 0xFFFF: the lane saw no row) to dv[q][col], col = chunk * 32 + ri (DenseMin).  The order
// statistics sample_select_kernel takes over these minima are >= those over every sample distance:
// tau_p (K-th + 1) still has K distinct rows below it, and tau_s only admits more rows (the recheck
// proves it per query either way).
// The minima are kept in float: v = pc(r) - 2 acc is one v_fma_f32 and the fold one v_min_f32 per
// register (exact: integers far below 2^24), a row past the chunk end contributes +inf.
template <bool ON, int MB>
struct DenseMin {  // the sample pass's lane minima (ON); empty in the thresholded passes
  float v[MB][16];
  __device__ __forceinline__ DenseMin() {
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int g = 0; g < 16; ++g) v[m][g] = __builtin_inff();
  }
  // v = pc(r) - 2 <q, r> of the 16 registers of M-block m (a row past the chunk end: no value)
  __device__ __forceinline__ void fold(const v16f& a, int m, int pc, bool ok) {
    const float pcf = ok ? (float)pc : __builtin_inff();
#pragma unroll
    for (int g = 0; g < 16; ++g) v[m][g] = fminf(v[m][g], fmaf(-2.0f, a[g], pcf));
  }
  // -> dv[q][col] as u16 (v + 1024; 0xFFFF: no row), col = chunk * 32 + lane row
  __device__ __forceinline__ void out(uint16_t* __restrict__ dv, int64_t dv_stride, int64_t col, int qbase, int h,
                                      int nq) const {
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int q = qbase + 32 * m + (g & 3) + 8 * (g >> 2) + 4 * h;
        if (q < nq)
          dv[(int64_t)q * dv_stride + col] = v[m][g] == __builtin_inff() ? (uint16_t)0xFFFF : (uint16_t)((int)v[m][g] + 1024);
      }
  }
};
template <int MB>
struct DenseMin<false, MB> {
  __device__ __forceinline__ void fold(const v16f&, int, int, bool) {}
  __device__ __forceinline__ void out(uint16_t*, int64_t, int64_t, int, int, int) const {}
};
template <int MODE, int MB>
__global__ __launch_bounds__(MWAVES * 64, 1) void hamming_mfma_kernel(
    const uint8_t* __restrict__ codes, int64_t n, int64_t row_begin, const uint8_t* __restrict__ queries, int nq,
    const int32_t* __restrict__ tau, uint64_t* __restrict__ cand, int32_t* __restrict__ ccnt, int capc,
    int64_t chunk_rows, int64_t chunk_stride, int64_t tile_stride, int nchunks, int nqb,
    const int32_t* __restrict__ rerun,
    const int32_t* __restrict__ qbflag, uint16_t* __restrict__ dv, int64_t dv_stride) {
  constexpr bool DENSE = MODE == MFMA_SAMPLE;
  constexpr int QPW = MfmaShape<MB>::QPW, QPB = MfmaShape<MB>::QPB;
  __shared__ __attribute__((aligned(16))) uint8_t smem[MfmaShape<MB>::SMEM];
  uint8_t* pk = smem;                                       // NPK packed tiles
  uint8_t* ub = smem + NPK * PKT;                           // NUB unpacked tiles
  int32_t* pcr = (int32_t*)(smem + NPK * PKT + NUB * UBT);  // NUB x 64 row popcounts
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int32_t* lcnt = pcr + NUB * RT + w * QPW;                 // this wave's list lengths
  int32_t* tq = pcr + NUB * RT + MWAVES * QPW + w * QPW;    // this wave's tau'(q) = tau(q) - pc(q)
  int32_t* stg = pcr + NUB * RT + 2 * MWAVES * QPW + w * (STG + 1);  // this wave's hit staging (+1 spare)

  const int l = lane_id();
  const int h = l >> 5, ri = l & 31;
  // XCD-aware bijective remap: consecutive logical blocks share one XCD's L2
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, q8 = nb >> 3, r8 = nb & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int chunk = L / nqb;
  const int qb = L - chunk * nqb;
  if (chunk >= nchunks) return;
  // re-run pass (exact fallback of the sampled threshold): only query blocks with a failed query
  if (qbflag && qbflag[qb] == 0) return;
#ifdef VRQ_K1M_STAMPS  // diagnostic build only (tools/probes/k1m_stamps.py): per-workgroup timeline
  const uint64_t st_start = __builtin_amdgcn_s_memrealtime();
#endif
  const int64_t row0 = row_begin + (int64_t)chunk * chunk_stride;
  // strided (sample pass): tile t starts at row0 + t * tile_stride, every tile whole (the plan keeps
  // the last one inside the corpus); otherwise the chunk is rows [row0, row0 + chunk_rows)
  const bool strided = tile_stride != RT;
  const int64_t row1 = strided ? n : (row0 + chunk_rows < n) ? row0 + chunk_rows : n;
  if (row0 >= row1) return;
  const int nrows = strided ? (int)chunk_rows : (int)(row1 - row0);
  const int ntiles = (nrows + RT - 1) / RT;

  // LDS-DMA of packed tile t: this wave's GPW pieces of 64 x 16 B (lane -> (row, piece) through the
  // swizzle).  Whole tiles take a uniform base + a fixed per-lane offset; the last partial tile
  // clamps each row to the chunk's last row.
  uint32_t doff[GPW];
#pragma unroll
  for (int i = 0; i < GPW; ++i) {
    const int p = (w * GPW + i) * 64 + l;
    const int r = p >> 3, c = (p & 7) ^ ((r >> 1) & 7);
    doff[i] = (uint32_t)(r * 128 + c * 16);
  }
  auto issue = [&](int t) __attribute__((always_inline)) {
    uint8_t* buf = pk + (t % NPK) * PKT;
    const int64_t tr0 = row0 + (int64_t)t * tile_stride;
    if (tr0 + RT <= row1) {
      const uint8_t* base = codes + tr0 * 128;
#pragma unroll
      for (int i = 0; i < GPW; ++i)
        __builtin_amdgcn_global_load_lds(base + doff[i], (__attribute__((address_space(3))) void*)(buf + (w * GPW + i) * 1024),
                                         16, 0, 0);
    } else {
#pragma unroll
      for (int i = 0; i < GPW; ++i) {
        int64_t row = tr0 + (doff[i] >> 7);
        row = row < row1 ? row : row1 - 1;
        __builtin_amdgcn_global_load_lds(codes + row * 128 + (doff[i] & 127),
                                         (__attribute__((address_space(3))) void*)(buf + (w * GPW + i) * 1024), 16, 0, 0);
      }
    }
  };
  const uint32_t pk0 = lds_addr(pk), ub0 = lds_addr(ub), pcr0 = lds_addr(pcr);
  const uint32_t lc0 = lds_addr(lcnt), stg0 = lds_addr(stg);
  // unit u of this wave = (nblk, piece) = ((4w+u) >> 3, (4w+u) & 7): lane -> tile row
  // 32*nblk + ri; piece p (dwords 4p..4p+3) holds k-steps 2p, 2p+1; lane-half h takes dword
  // 4p+2h of step 2p and 4p+2h+1 of step 2p+1 (one 8-byte read per lane).  Unpacked layout
  // [n-block][k-step][lane][16 B]: group g = 16*nblk + s.
  uint32_t usrc[4], udst[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int unit = 4 * w + u, nblk = unit >> 3, p = unit & 7;
    const int r = nblk * 32 + ri;
    usrc[u] = (uint32_t)(pk_slot(r, p) * 16 + h * 8);
    udst[u] = (uint32_t)(((nblk * KS + 2 * p) * 64 + l) * 16);
  }
  // row popcounts: tile rows 16w..16w+15, 4 lanes per row, 2 pieces each
  const int pr = 16 * w + (l >> 2), pc0 = 2 * (l & 3);
  const uint32_t psrc0 = (uint32_t)(pk_slot(pr, pc0) * 16), psrc1 = (uint32_t)(pk_slot(pr, pc0 + 1) * 16);
  auto unpack_write = [&](const v2i& v, int u, uint32_t ubuf) __attribute__((always_inline)) {
    lds_write128(ubuf + udst[u], unpack_row32((uint32_t)v.x));
    lds_write128(ubuf + udst[u] + 1024, unpack_row32((uint32_t)v.y));
  };
  auto rowpc_write = [&](const v4i& a, const v4i& c, uint32_t pbuf) __attribute__((always_inline)) {
    int pc = (__popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w)) +
             (__popc(c.x) + __popc(c.y) + __popc(c.z) + __popc(c.w));
    pc += __builtin_amdgcn_update_dpp(0, pc, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    pc += __builtin_amdgcn_update_dpp(0, pc, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    if ((l & 3) == 0) lds_write32(pbuf + (uint32_t)(pr * 4), pc);
  };

  // ---- prologue: DMA tiles 0..NPK-1, A fragments + thresholds, unpack tiles 0 and 1 ----
  for (int t = 0; t < NPK && t < ntiles; ++t) issue(t);

  const int qbase = qb * QPB + w * QPW;
  v4i A[MB][KS];  // [m][s]: bits 64s+32h .. +31 of query qbase + 32m + ri as 32 e2m1 values
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int q = qbase + 32 * m + ri;
    const bool qok = q < nq && (!rerun || rerun[q]);
    const uint4* qp = reinterpret_cast<const uint4*>(queries + (int64_t)(qok ? q : 0) * 128);
    int pc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 v = qp[c];
      const uint32_t wd[4] = {qok ? v.x : 0u, qok ? v.y : 0u, qok ? v.z : 0u, qok ? v.w : 0u};
      pc += __popc(wd[0]) + __popc(wd[1]) + __popc(wd[2]) + __popc(wd[3]);
      A[m][2 * c] = unpack_query32(h ? wd[2] : wd[0]);
      A[m][2 * c + 1] = unpack_query32(h ? wd[3] : wd[1]);
    }
    // tau'(q) = tau(q) - pc(q): a row is a candidate iff pc(r) - 2<q,r> < tau'
    if (h == 0) tq[32 * m + ri] = DENSE ? 0 : qok ? tau[q] - pc : -0x40000000;  // padded queries never accept
  }
  // A lives in the accumulator file (the MFMA reads it from there); VGPRs hold the
  // accumulators, seeds and the B ring
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+a"(A[m][s]));
  // accumulator seed tau'/2 per register (register g of lane half h holds query
  // (g&3) + 8(g>>2) + 4h of the M-block): after the K loop acc = <q,r> + tau'/2, and the row is
  // a candidate iff pc(r) - 2<q,r> < tau'  <=>  acc > pc(r)/2.  The seeds of M-block m stay in LDS
  // (sd: [m][h][g] floats, 64 B per lane half: broadcast reads) and are loaded into the
  // accumulators of an n-block right after that block's epilogue.
  float* sd = reinterpret_cast<float*>(pcr + NUB * RT + 2 * MWAVES * QPW + MWAVES * (STG + 1)) + w * MB * 32;
#pragma unroll
  for (int m = 0; m < MB; ++m)
    if (l < 32) {  // lane l writes [m][h = l >> 4][g = l & 15]
      const int g = l & 15, hh = l >> 4;
      sd[m * 32 + l] = 0.5f * (float)tq[32 * m + (g & 3) + 8 * (g >> 2) + 4 * hh];
    }
  const uint32_t sd0 = lds_addr(sd) + (uint32_t)(h * 64);  // this lane half's 16 seeds of M-block 0
  auto load_seed = [&](v16f& a, int m) __attribute__((always_inline)) {
    v4i p0, p1, p2, p3;
    lds_read128(p0, sd0 + (uint32_t)(m * 128));
    lds_read128(p1, sd0 + (uint32_t)(m * 128 + 16));
    lds_read128(p2, sd0 + (uint32_t)(m * 128 + 32));
    lds_read128(p3, sd0 + (uint32_t)(m * 128 + 48));
    const v16i x = __builtin_shufflevector(__builtin_shufflevector(p0, p1, 0, 1, 2, 3, 4, 5, 6, 7),
                                           __builtin_shufflevector(p2, p3, 0, 1, 2, 3, 4, 5, 6, 7), 0, 1, 2, 3, 4,
                                           5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    a = __builtin_bit_cast(v16f, x);
  };
  for (int i = l; i < QPW; i += 64) lcnt[i] = 0;
  __syncthreads();
  // at most k tiles' DMA still in flight (k <= NPK - 2; wave-uniform k)
  auto wait_tiles = [&](int k) __attribute__((always_inline)) {
    if (k <= 0) wait_vm<0>();
    else if (k == 1) wait_vm<GPW>();
    else if (k == 2) wait_vm<2 * GPW>();
    else if (k == 3) wait_vm<3 * GPW>();
    else wait_vm<4 * GPW>();
  };
  static_assert(NPK - 2 <= 4, "wait_tiles covers up to 4 tiles in flight");
  const int nissued = ntiles < NPK ? ntiles : NPK;
  wait_tiles(nissued - 2);
  barrier_all();  // packed tiles 0 and 1 visible to all waves
  {
    v2i pv[8];
    v4i pa[2], pb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int u = 0; u < 4; ++u) lds_read64(pv[4 * t + u], pk0 + (uint32_t)(t * PKT) + usrc[u]);
      lds_read128(pa[t], pk0 + (uint32_t)(t * PKT) + psrc0);
      lds_read128(pb[t], pk0 + (uint32_t)(t * PKT) + psrc1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(pv[0]), "+v"(pv[1]), "+v"(pv[2]), "+v"(pv[3]), "+v"(pv[4]), "+v"(pv[5]), "+v"(pv[6]),
                   "+v"(pv[7]), "+v"(pa[0]), "+v"(pa[1]), "+v"(pb[0]), "+v"(pb[1])::"memory");
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int u = 0; u < 4; ++u) unpack_write(pv[4 * t + u], u, ub0 + (uint32_t)(t * UBT));
      rowpc_write(pa[t], pb[t], pcr0 + (uint32_t)(t * RT * 4));
    }
  }
  wait_tiles(nissued - 3);
  wait_lgkm0();

  // ---- hit path ----
  const int64_t qstride = (int64_t)nchunks * capc;
  // this wave's lists: query qbase + ql, chunk `chunk` -> cbase + ql * qstride + pos
  uint64_t* const cbase = cand + ((int64_t)qbase * nchunks + chunk) * capc;
  int nst = 0;  // staged entries (wave-uniform)
  // Staged entries -> per-(query, chunk) lists in HBM.  The first 64 entries of a tile go
  // asynchronously: read back from the stage in group 20 + MB (all hits of a tile are staged by
  // group 19 + MB), list positions taken by ds_add_rtn in group 24 + MB, both in the MFMA shadow; the global
  // stores issue at the top of the next iteration, BEFORE that iteration's LDS-DMA, so the
  // end-of-tile vmcnt wait never waits on a store issued after a DMA.  Entries past 64 (and a
  // stage overflow) take the synchronous path at the end of the tile.
  int fe = 0, fpos = 0, nfl = 0;
  int64_t fbase = 0;
  auto fkey = [&](int e, int64_t base_row) __attribute__((always_inline)) {
    return ((uint64_t)(uint32_t)(e >> ENT_V_SHIFT) << KEY_ROW_BITS) | (uint64_t)(base_row + (e & 127));
  };
  auto store_flushed = [&]() __attribute__((always_inline)) {
    if (nfl) {
      const int ql = (fe >> ENT_Q_SHIFT) & 127;
#ifndef VRQ_K1M_PROBE_NOSTORE  // timing-only probe builds (lists left incomplete)
      if (l < nfl && fpos < capc) cbase[ql * qstride + fpos] = fkey(fe, fbase);
#endif
      nfl = 0;
    }
  };
  auto flush_from = [&](int i_begin, int64_t base_row) __attribute__((always_inline)) {
    if (nst > STG) {  // staging overflowed in this tile: every list of the wave -> exact rescan
      for (int i = l; i < QPW; i += 64) lds_add32(lc0 + (uint32_t)(i * 4), capc + 1);
      nst = STG;
    }
    for (int i0 = i_begin; i0 < nst; i0 += 64) {
      const int i = i0 + l;
      int e = 0, pos = 0;
      if (i < nst) lds_read32(e, stg0 + (uint32_t)(i * 4));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(e)::"memory");
      const int ql = (e >> ENT_Q_SHIFT) & 127;
      if (i < nst) lds_add_rtn32(pos, lc0 + (uint32_t)(ql * 4), 1);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pos)::"memory");
      if (i < nst && pos < capc) cbase[ql * qstride + pos] = fkey(e, base_row);
    }
    nst = 0;
  };
  // hits of block (m, n-block) whose rows are rel7 = row - (t-1)*64.  Blocks without a hit stop at
  // the max3 tree + one compare; a block with hits (rare: ~0.5 % of blocks at 100M rows) takes one
  // ballot per register (few live registers: this path is inlined into the MFMA loop).  Positions
  // past STG land in a spare slot and the flush marks the whole wave's lists overflowed (exact rescan).
  auto block_hits = [&](const v16f& a, int m, int pc, float hp, int rel7) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const uint64_t mask = __ballot(a[g] > hp);
      if (mask) {
        if ((mask >> l) & 1) {
          const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
          // lane-dependent values of this rare path are derived from an opaque copy of the lane
          // id, so loop-invariant code motion cannot hoist them into registers held by the loop
          int lo = l;
          asm volatile("" : "+v"(lo));
          const int ql = 32 * m + (g & 3) + 8 * (g >> 2) + 4 * (lo >> 5);
          // acc = <q,r> + tau'/2 with tau' = tau(q) - pc(q), so pc(r) - 2 acc = dist - tau(q) in
          // [-1025, -1] for a hit (exact integers): no per-query value to fetch on this path
          const int v = pc - (int)(2.0f * a[g]);
          const int pos = nst + below < STG ? nst + below : STG;
          lds_write32(stg0 + (uint32_t)(pos * 4), ((v + ENT_V_BIAS) << ENT_V_SHIFT) | (ql << ENT_Q_SHIFT) | (rel7 - ri + (lo & 31)));
        }
        nst += __popcll(mask);
      }
    }
  };
  // Branch-light form: per lane a 16-bit mask of its registers above the threshold; when no lane
  // holds two hits (one ballot proves it) each hit lane stages one entry -- its single hit is its
  // largest register (the others are <= hp), found by a max3 tree, its query row by the mask's
  // lowest bit -- at its rank among the hit lanes.  Otherwise the 16-ballot walk above.
  auto block_hits_fast = [&](const v16f& a, int m, int pc, float hp, int rel7) __attribute__((always_inline)) {
    uint32_t m16 = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) m16 |= (a[g] > hp ? 1u : 0u) << g;
#ifdef VRQ_K1M_PROBE_NOSLOW  // timing-only probe builds (wrong lists when a lane holds two hits)
    if (false) {
#else
    if (__ballot((m16 & (m16 - 1)) != 0)) {  // some lane holds two or more hits (rare)
#endif
      block_hits(a, m, pc, hp, rel7);
    } else {
      const uint64_t lanes = __ballot(m16 != 0);
      if (m16) {
        const v16i b = __builtin_bit_cast(v16i, a);  // >= 0 patterns order like their floats
        const int x0 = max(max(b[0], b[1]), b[2]), x1 = max(max(b[3], b[4]), b[5]), x2 = max(max(b[6], b[7]), b[8]);
        const int x3 = max(max(b[9], b[10]), b[11]), x4 = max(max(b[12], b[13]), b[14]);
        const float mx = __int_as_float(max(max(max(x0, x1), x2), max(max(x3, x4), b[15])));
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(lanes >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)lanes, 0));
        int lo = l;
        asm volatile("" : "+v"(lo));
        const int g = __builtin_ctz(m16);
        const int ql = 32 * m + (g & 3) + 8 * (g >> 2) + 4 * (lo >> 5);
        const int v = pc - (int)(2.0f * mx);
        const int pos = nst + below < STG ? nst + below : STG;
        lds_write32(stg0 + (uint32_t)(pos * 4), ((v + ENT_V_BIAS) << ENT_V_SHIFT) | (ql << ENT_Q_SHIFT) | (rel7 - ri + (lo & 31)));
      }
      nst += __popcll(lanes);
    }
  };
  auto row_pc = [&](int pcv, int lr) __attribute__((always_inline)) {  // past the end: no hit
    return lr < nrows ? pcv : 0x40000000;
  };
  // DENSE: the 16 values v = dist - pc(q) of block (m, n-block) (row lr of the chunk) fold into this
  // lane's running minima; only those leave the kernel (dense_out)
  DenseMin<DENSE, MB> dmin;
  auto block_dense = [&](const v16f& a, int m, int pc, int lr) __attribute__((always_inline)) {
    dmin.fold(a, m, pc, lr < nrows);
  };

  // ---- main loop: 32 groups per tile (schedule above) ----
  v4i ring[NRING];
  const uint32_t bl0 = ub0 + (uint32_t)(l * 16);  // + tile slot + group * 1024: this lane's B fragment
  int pcvP = 0;  // previous tile's n-block 1 row popcount
  uint64_t hitm[MB];  // per M-block: lanes of the previous n-block with a candidate (wave-uniform)
#pragma unroll
  for (int m = 0; m < MB; ++m) hitm[m] = 0;
  int hpb = 0;   // the previous n-block's per-lane threshold pc(r)/2, as float bits
  v16f acc[2][MB];  // [n-block][m]
  if constexpr (!DENSE)
    static_for<0, MB>([&](auto M) {
      constexpr int m = decltype(M)::value;
      load_seed(acc[0][m], m);
      load_seed(acc[1][m], m);
    });
  barrier_all();  // B_0: unpacked tiles 0 and 1, packed tile 2 visible
#ifdef VRQ_K1M_STAMPS
  const uint64_t st_loop = __builtin_amdgcn_s_memrealtime();
#endif
  static_for<0, BAHEAD>([&](auto G) {
    constexpr int g = decltype(G)::value;
    lds_read128_imm<g * 1024>(ring[g], bl0);
  });
  // ntiles >= 1 (row0 < row1 above): no zero-trip path on which the seed and B-fragment reads issued
  // above would stay in flight into the epilogue (tests/isa_check.py follows every static path)
  __builtin_assume(ntiles > 0);
  int st_prev = 0;  // VRQ_K1M_DMA_AHEAD: the previous iteration issued list stores
  (void)st_prev;
  for (int t = 0; t < ntiles; ++t) {
#if VRQ_K1M_DMA_AHEAD
    // the packed slot of tile t+1 is free once tile t+1 was unpacked (iteration t-1): tile t+5 goes there
    // now, one iteration earlier than a refill of tile t's own slot (iteration 0 also issues tile 4 into
    // tile 0's slot, unpacked in the prologue) -- two tile-times of DMA lead for the end-of-tile wait
    const int st_now = nfl != 0 ? 1 : 0;  // wave-uniform: this iteration issues list stores
    store_flushed();                       // previous tile's first 64 hits
    if (t == 0 && NPK < ntiles) issue(NPK);
    if (t + NPK + 1 < ntiles) issue(t + NPK + 1);
#else
    store_flushed();                       // previous tile's first 64 hits
    if (t + NPK < ntiles) issue(t + NPK);  // into the slot of tile t (unpacked in iteration t-2)
#endif
    const uint32_t blt = bl0 + (uint32_t)((t % NUB) * UBT);
    const uint32_t bln = bl0 + (uint32_t)(((t + 1) % NUB) * UBT);
    const uint32_t ubw = ub0 + (uint32_t)(((t + 2) % NUB) * UBT);
    const uint32_t pks = pk0 + (uint32_t)(((t + 2) % NPK) * PKT);
    int pcv[2];
    lds_read32(pcv[0], pcr0 + (uint32_t)(((t % NUB) * RT + ri) * 4));
    lds_read32(pcv[1], pcr0 + (uint32_t)(((t % NUB) * RT + 32 + ri) * 4));
    v2i pv;
    v4i pa, pb;
    VRQ_SCHED_FENCE();
    static_for<0, NG>([&](auto GI) {
      constexpr int gi = decltype(GI)::value;
      constexpr int nbk = gi >> 4, s = gi & 15, j = gi & 15;
      if constexpr (gi + BAHEAD < NG)
        lds_read128_imm<(gi + BAHEAD) * 1024>(ring[(gi + BAHEAD) & (NRING - 1)], blt);
      else
        lds_read128_imm<(gi + BAHEAD - NG) * 1024>(ring[(gi + BAHEAD) & (NRING - 1)], bln);
      // packed reads of the unpack units (used 5 groups later) and of the row popcounts
      if constexpr ((gi & 7) == 1) lds_read64(pv, pks + usrc[gi >> 3]);
      if constexpr (gi == 12) {
        lds_read128(pa, pks + psrc0);
        lds_read128(pb, pks + psrc1);
      }
      // every LDS operation issued up to the B read of group gi - BAHEAD has completed (k1m_wait): the
      // fragment of this group, the packed unit read 5 groups ago, the popcounts, the seeds
      asm volatile("s_waitcnt lgkmcnt(%7)"
                   : "+v"(ring[gi & (NRING - 1)]), "+v"(pv), "+v"(pcv[0]), "+v"(pcv[1]), "+v"(pa), "+v"(pb), "+v"(fe)
                   : "n"(k1m_wait(gi, MB, DENSE))
                   : "memory");
      // The group's non-MFMA work is cut into four slots that sit between its MFMAs (slot k after
      // MFMA k; at MB = 2 slots 2k and 2k+1 after MFMA k): an in-order wave issues them while the
      // matrix core runs, at most ~3 vector instructions per slot, instead of one burst after the
      // last MFMA of the group.  Per group kind:
      //   hit test of M-block m (j = 2+m): max3 pairs in slots 0-2, the last max3 + compare in 3
      //   the n-block threshold pc(r)/2 (j = 1), the (rare) hit-extraction branch (j = 3+MB, slot 3)
      //   unpack of unit u (gi = 8u+6): 3 + 2 ops per dword, the two LDS writes in slots 1 and 3
      //   row popcounts (gi = 28): 4 + 4 bcnt, the lane-quad sums, the LDS write
      //   accumulator re-seeds (j = 4+MB .. 3+2MB... one M-block per group, one read per slot)
      //   asynchronous hit flush (gi = 20+MB and 24+MB, slot 3)
      constexpr bool TEST = !DENSE && j >= 2 && j < 2 + MB;
      constexpr int tm = TEST ? j - 2 : 0;
      constexpr bool UNPACK = (gi & 7) == 6;
      constexpr bool SEED = !DENSE && j >= 4 + MB && j < 4 + 2 * MB;
      constexpr int sm = SEED ? j - 4 - MB : 0;
      int e0 = 0, e1 = 0, e2 = 0, e3 = 0, e4 = 0, f0 = 0;
      uint32_t u0 = 0, u1 = 0, u2 = 0;
      int pc0 = 0, pc1 = 0;
      auto slot = [&](auto K) __attribute__((always_inline)) {
        constexpr int k = decltype(K)::value;
        const v16i bb = __builtin_bit_cast(v16i, acc[nbk ^ 1][tm]);
        if constexpr (TEST) {
          if constexpr (k == 0) {
            e0 = max(max(bb[0], bb[1]), bb[2]);
            e1 = max(max(bb[3], bb[4]), bb[5]);
            asm volatile("" ::"v"(e0), "v"(e1));
          } else if constexpr (k == 1) {
            e2 = max(max(bb[6], bb[7]), bb[8]);
            e3 = max(max(bb[9], bb[10]), bb[11]);
            asm volatile("" ::"v"(e2), "v"(e3));
          } else if constexpr (k == 2) {
            e4 = max(max(bb[12], bb[13]), bb[14]);
            f0 = max(max(e0, e1), e2);
            asm volatile("" ::"v"(e4), "v"(f0));
          } else {
            hitm[tm] = __ballot(max(max(e3, e4), max(bb[15], f0)) > hpb);
          }
        }
        if constexpr (!DENSE && j == 1 && k == 0) {
          // the n-block's threshold pc(r)/2 as float bits (>= 0); no previous n-block before tile 0:
          // a threshold no accumulator exceeds
          const int pcr_ = nbk == 0 ? pcvP : pcv[0];
          const int lr = (nbk == 0 ? (t - 1) * RT + 32 : t * RT) + ri;
          hpb = (nbk == 0 && t == 0) ? 0x7fffffff : __float_as_int(0.5f * (float)row_pc(pcr_, lr));
          asm volatile("" : "+v"(hpb));
        }
        if constexpr (UNPACK) {  // unpack_row32 of pv.x (slots 0, 1) and pv.y (slots 2, 3)
          constexpr int half = k >> 1;
          const uint32_t wv = (uint32_t)(half ? pv.y : pv.x);
          if constexpr ((k & 1) == 0) {
            u0 = wv & 0x11111111u;
            u1 = wv & 0x22222222u;
            u2 = wv & 0x44444444u;
            asm volatile("" ::"v"(u0), "v"(u1), "v"(u2));
          } else {
            v4i r;
            r.x = (int)u0;
            r.y = (int)u1;
            r.z = (int)u2;
            r.w = (int)((wv >> 1) & 0x44444444u);
            lds_write128(ubw + udst[gi >> 3] + (uint32_t)(half * 1024), r);
          }
        }
        if constexpr (gi == 28) {  // row popcounts of tile t+2
          if constexpr (k == 0) {
            pc0 = __popc(pa.x) + __popc(pa.y) + __popc(pa.z) + __popc(pa.w);
            asm volatile("" ::"v"(pc0));
          } else if constexpr (k == 1) {
            pc1 = __popc(pb.x) + __popc(pb.y) + __popc(pb.z) + __popc(pb.w);
            asm volatile("" ::"v"(pc1));
          } else if constexpr (k == 2) {
            pc0 = pc0 + pc1;
            pc0 += __builtin_amdgcn_update_dpp(0, pc0, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
            asm volatile("" ::"v"(pc0));
          } else {
            pc0 += __builtin_amdgcn_update_dpp(0, pc0, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
            // every lane of the quad writes the same sum (no exec-masked branch: the counted waits
            // above assume this write is issued on every path)
            lds_write32(pcr0 + (uint32_t)(((t + 2) % NUB) * RT * 4 + pr * 4), pc0);
          }
        }
        if constexpr (SEED) {  // one 16-byte piece of M-block sm's seeds per slot, into its accumulator
          v4i piece;
          lds_read128(piece, sd0 + (uint32_t)(sm * 128 + k * 16));
          v16i x = __builtin_bit_cast(v16i, acc[nbk ^ 1][sm]);
          x[4 * k] = piece.x;
          x[4 * k + 1] = piece.y;
          x[4 * k + 2] = piece.z;
          x[4 * k + 3] = piece.w;
          acc[nbk ^ 1][sm] = __builtin_bit_cast(v16f, x);
        }
        if constexpr (DENSE && j >= 2 && j < 2 + MB && k == 0) {
          if (nbk == 1 || t > 0) {
            const int pcr_ = nbk == 0 ? pcvP : pcv[0];
            const int lr = (nbk == 0 ? (t - 1) * RT + 32 : t * RT) + ri;
            block_dense(acc[nbk ^ 1][j - 2], j - 2, pcr_, lr);
          }
        }
        if constexpr (k == 3) {
          // async flush, step 1 (after the last hit extraction of the tile, group 16 + 3 + MB): the
          // stage's first 64 entries; step 2, four groups (>= 4 LDS operations) later: list positions
          if constexpr (gi == 20 + MB && !DENSE) {
            lds_read32(fe, stg0 + (uint32_t)(l * 4));
            nfl = nst < 64 ? nst : 64;
          }
          if constexpr (gi == 24 + MB && !DENSE)  // step 2 (idle lanes add 0)
            lds_add_rtn32(fpos, lc0 + (uint32_t)(((fe >> ENT_Q_SHIFT) & 127) * 4), l < nfl ? 1 : 0);
          // hit extraction of the previous n-block's flagged M-blocks, once per n-block (rare)
          if constexpr (!DENSE && j == 3 + MB) {
            // (hitm[m] is assigned by every n-block's test of M-block m before this point)
            uint64_t any = hitm[0];
#pragma unroll
            for (int m = 1; m < MB; ++m) any |= hitm[m];
            if (any) {
              const int pcr_ = nbk == 0 ? pcvP : pcv[0];
              const int lr = (nbk == 0 ? (t - 1) * RT + 32 : t * RT) + ri;
              const int pc = row_pc(pcr_, lr);
              const float hp = 0.5f * (float)pc;
              static_for<0, MB>([&](auto M) {
                constexpr int mm = decltype(M)::value;
#ifndef VRQ_K1M_PROBE_NOHITS  // timing-only probe builds: no hit extraction at all
                if (hitm[mm]) block_hits_fast(acc[nbk ^ 1][mm], mm, pc, hp, (nbk == 0 ? 32 : 64) + ri);
#endif
              });
            }
          }
        }
      };
      static_for<0, MB>([&](auto M) {
        constexpr int m = decltype(M)::value;
        if constexpr (s == 0 && !DENSE)  // the seeds loaded after the block's last epilogue have landed
          asm volatile("" : "+v"(acc[nbk][m]));
        acc[nbk][m] = mfma_fp4(A[m][s], ring[gi & (NRING - 1)], (s == 0 && DENSE) ? v16f{} : acc[nbk][m]);
        // pin the accumulator here: the MFMA intrinsics are pure, and without a use at this
        // point IR-level sinking moves them past the scheduling fences
        asm volatile("" : "+v"(acc[nbk][m]));
        VRQ_SCHED_FENCE();
        if constexpr (MB == 4) {
          slot(std::integral_constant<int, m>{});
        } else {
          slot(std::integral_constant<int, 2 * m>{});
          slot(std::integral_constant<int, 2 * m + 1>{});
        }
        VRQ_SCHED_FENCE();
      });
      VRQ_SCHED_FENCE();
    });
    pcvP = pcv[1];
    // packed tile t+3 (unpacked next iteration) landed; this wave's LDS writes done
    {
#ifndef VRQ_K1M_PROBE_NOVMWAIT  // timing-only probe builds (wrong results)
#if VRQ_K1M_DMA_AHEAD
      // issued after tile t+3's DMA: the k tiles after it and the list stores of this iteration and the
      // previous one (each store instruction sits before its iteration's DMA; rare-path stores are drained)
      const int last = t + NPK + 1 < ntiles ? t + NPK + 1 : ntiles - 1;
      const int k = last - (t + 3), ns = st_prev + st_now;
      if (k <= 0) wait_vm<0>();
      else if (k == 1) {
        if (ns == 0) wait_vm<GPW>(); else if (ns == 1) wait_vm<GPW + 1>(); else wait_vm<GPW + 2>();
      } else {
        if (ns == 0) wait_vm<2 * GPW>(); else if (ns == 1) wait_vm<2 * GPW + 1>(); else wait_vm<2 * GPW + 2>();
      }
      st_prev = st_now;
#else
      const int last = t + NPK < ntiles ? t + NPK : ntiles - 1;  // last tile issued so far
      wait_tiles(last - (t + 3));
#endif
#endif
    }
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(fpos), "+v"(fe)::"memory");
    fbase = row0 + (int64_t)(t - 1) * RT;
    if (nst > 64) {  // rare: more than 64 hits in one tile
      flush_from(64, fbase);
      if (VRQ_K1M_DMA_AHEAD) wait_vm<0>();  // (drained: the next waits count only the per-tile stores)
    }
    nst = 0;
#ifndef VRQ_K1M_PROBE_NOBARRIER  // timing-only probe builds (wrong results)
    barrier_all();  // B_{t+1}
#endif
  }
  store_flushed();
  if (ntiles > 0) {  // n-block 1 of the last tile
    const int lr = (ntiles - 1) * RT + 32 + ri;
    const int pc = row_pc(pcvP, lr);
    const float hp = 0.5f * (float)pc;
    static_for<0, MB>([&](auto M) {
      constexpr int m = decltype(M)::value;
      if constexpr (DENSE)
        block_dense(acc[1][m], m, pcvP, lr);
      else
        if (any_above(acc[1][m], hp)) block_hits_fast(acc[1][m], m, pc, hp, 96 + ri);  // rel7 against tile ntiles-2
    });
    if (nst) flush_from(0, row0 + (int64_t)(ntiles - 2) * RT);
  }
  wait_lgkm0();
#ifdef VRQ_K1M_STAMPS
  if (!DENSE && threadIdx.x == 0) {  // the MAIN pass gets the workspace head as `dv` in this build
    uint64_t* stp = reinterpret_cast<uint64_t*>(dv) + 4 * (int64_t)L;
    stp[0] = st_start;
    stp[1] = st_loop;
    stp[2] = __builtin_amdgcn_s_memrealtime();
    stp[3] = ((uint64_t)__builtin_amdgcn_s_getreg(63508) << 32) | (uint32_t)__builtin_amdgcn_s_getreg(63492);
  }
#endif
  if constexpr (DENSE)
    dmin.out(dv, dv_stride, (int64_t)chunk * 32 + ri, qbase, h, nq);
  else
    for (int i = l; i < QPW; i += 64) {
      const int q = qbase + i;
      if (q < nq && (!rerun || rerun[q])) ccnt[(int64_t)q * nchunks + chunk] = lcnt[i];
    }
}

// ---------------------------------------------------------------------------------------------
// K1s: the thresholded pass of large batches (nq >= 512) with the roles of queries and rows swapped.
//
// K1m keeps the queries in the accumulator file and streams 64-row tiles through a shared LDS ring:
// every tile costs an LDS-DMA, a shared unpack, a workgroup barrier and 32 KiB of B-fragment reads per
// wave.  Here each wave keeps a ROW SET of SRB x 32 corpus rows resident as the MFMA A operand (SRB x
// 64 AGPRs, unpacked once per row set) and streams the workgroup's 512 queries from LDS as packed bits
// (64 KiB, loaded once per workgroup), unpacking each query k-step with 5 VALU ops:
//   * per 32-query block: 16 k-steps x SRB MFMAs (32x32x64 FP4), each B fragment (one dword per lane)
//     feeding SRB MFMAs; 4 ds_read_b128 of queries per block and wave; no LDS writes and no barrier
//     inside the loop;
//   * each of the SNW waves owns every SNW-th row set of the workgroup's chunk and LDS-DMAs the next one
//     into its own staging buffer (SRB x 4 KiB) a whole row set (16 query blocks) ahead;
//   * lane (j, h) of a 32x32 accumulator holds query j of the block and rows (g&3) + 8(g>>2) + 4h of
//     the row block.  Seeds 1024 - pc(r)/2 (per register, from LDS) make acc = 1024 + <q,r> - pc(r)/2,
//     always > 0 for a row of the chunk (-4096 seeds mask the rows past its end), so the candidate
//     test dist < tau(q)  <=>  acc > thr(q) = 1024 + (pc(q) - tau(q))/2  is a max3 tree over the float
//     bit patterns and one compare per lane against its query's threshold (thr > 0: tau <= 1025);
//     v = dist - tau(q) = 2 thr - 2 acc exactly;
//   * the test of a block's accumulators runs in the next block's MFMA shadow (two accumulator sets);
//     hits are staged per wave and appended to the per-(query, chunk) lists at positions taken from the
//     workgroup's per-query LDS counters (the waves share the chunk), once per row set.  The stage holds
//     the set's query blocks' hits in block order, so a stage overflow marks only the lists of the
//     blocks from the first one that went past its end (exact rescan), not all 512 queries' (ADVICE
//     round 5; a flush check after every block cost the config-2 pass 2 %).
// Two instances:
//   * <SRB = 2, SNW = 8>: two waves per SIMD (256 registers each; 64-row sets); at the row-set switch a
//     wave rebuilds its A fragments and seeds from the staging buffer while the SIMD's other wave runs.
//   * <SRB = 4, SNW = 4>: one wave per SIMD (A = all 256 AGPRs; 128-row sets): each query fragment feeds
//     4 MFMAs (half the unpack VALU and query reads per MFMA) and the row-set switch is spread over the
//     last query block of the set -- k-step s's new A fragments are unpacked right after that k-step's
//     MFMAs, from staging reads issued one block ahead -- so the matrix core does not wait for it.
// The lists, their keys and the suffix merge are K1m's, so the pass is a drop-in for K1m's MB = 4
// instance (same launch geometry: one workgroup per (chunk, 512-query block)).
// K1s takes the large-batch pass up to this many (query, row) pairs per launch (1M rows x 1024 queries:
// 0.34 vs 0.39 ms, config-2 step 0.538 vs 0.583 ms; 4M: 1.25 vs 1.36 ms).  Above, K1m: two waves per
// SIMD each unpacking every query fragment cost more energy per MFMA than K1m's shared tile, and a long
// pass is power-bound -- 100M x 1024 in the config-4 bench ran 32.8 ms on K1s vs 31.0 on K1m on one box
// (K1s 2.22 GHz / 0.75 of the matrix cores busy vs K1m 2.37 GHz / 0.71; profiles/r5_k1s_ab.jsonl).
constexpr double kSwapMaxPairs = 4294967296.0;
// A/B builds only (tools/build_variants.sh -D...): VRQ_K1S_LARGE=1 runs passes above kSwapMaxPairs on
// K1s<4, 4> instead of K1m; VRQ_K1S_RB4=1 runs the shorter ones on K1s<4, 4> instead of K1s<2, 8>
#ifndef VRQ_K1S_LARGE
#define VRQ_K1S_LARGE 0
#endif
#ifndef VRQ_K1S_RB4
#define VRQ_K1S_RB4 0
#endif

constexpr int SQPB = 512;  // queries per workgroup (16 blocks of 32)
template <int SRB, int SNW>
struct SwapShape {
  static constexpr int SRS = SRB * 32;      // rows per row set
  static constexpr int QBYTES = SQPB * 128;  // packed queries (swizzled 16-B pieces)
  static constexpr int RBYTES = SRS * 128;   // one wave's row staging
  static constexpr int SMEM = QBYTES + SNW * RBYTES + SQPB * 4 /* thr */ + SQPB * 4 /* list lengths */ +
                              SNW * (STG + 1) * 4 + SNW * SRB * 32 * 4 /* seeds */;
  static_assert(SMEM <= 160 * 1024, "LDS budget");
  static_assert(SRS <= 128, "a staged entry keeps 7 bits of row in the row set");
  static_assert((SRB == 2 && SNW == 8) || (SRB == 4 && SNW == 4), "the two instances");
};
// staged hit entry of K1s (u32): (v + 1025) << 16 | query-in-workgroup << 7 | row in the row set
constexpr int SENT_V_SHIFT = 16, SENT_Q_SHIFT = 7;

template <int MODE, int SRB, int SNW>
__global__ __launch_bounds__(SNW * 64, 1) void hamming_mfma_swap_kernel(
    const uint8_t* __restrict__ codes, int64_t n, int64_t row_begin, const uint8_t* __restrict__ queries, int nq,
    const int32_t* __restrict__ tau, uint64_t* __restrict__ cand, int32_t* __restrict__ ccnt, int capc,
    int64_t chunk_rows, int64_t chunk_stride, int64_t tile_stride, int nchunks, int nqb,
    const int32_t* __restrict__ rerun, const int32_t* __restrict__ qbflag, uint16_t* __restrict__ dv,
    int64_t dv_stride) {
  static_assert(MODE == MFMA_MAIN || MODE == MFMA_RERUN, "thresholded passes only");
  using Sh = SwapShape<SRB, SNW>;
  constexpr int SRS = Sh::SRS;
#ifndef VRQ_K1S_SPREAD
#define VRQ_K1S_SPREAD 1
#endif
  constexpr bool SPREAD = SNW == 4 && VRQ_K1S_SPREAD;  // one wave per SIMD: the switch is spread over a block
  __shared__ __attribute__((aligned(16))) uint8_t smem[Sh::SMEM];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* qpk = smem;
  uint8_t* rst = smem + Sh::QBYTES + w * Sh::RBYTES;  // this wave's row staging
  float* thr = reinterpret_cast<float*>(smem + Sh::QBYTES + SNW * Sh::RBYTES);
  int32_t* lcnt = reinterpret_cast<int32_t*>(thr + SQPB);
  int32_t* stg = lcnt + SQPB + w * (STG + 1);
  float* sdw = reinterpret_cast<float*>(lcnt + SQPB + SNW * (STG + 1)) + w * SRB * 32;
  const int l = lane_id();
  const int h = l >> 5, ri = l & 31;
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, q8 = nb >> 3, r8 = nb & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int chunk = L / nqb;
  const int qb = L - chunk * nqb;
  if (chunk >= nchunks) return;
  if (qbflag && qbflag[qb] == 0) return;
  const int64_t row0 = row_begin + (int64_t)chunk * chunk_stride;
  const int64_t row1 = (row0 + chunk_rows < n) ? row0 + chunk_rows : n;
  if (row0 >= row1) return;
  const int nrs = (int)((row1 - row0 + SRS - 1) / SRS);  // row sets of the chunk; wave w takes w, w + SNW, ...
  const int qbase = qb * SQPB;
  const int nqv = nq - qbase < SQPB ? nq - qbase : SQPB;
  const int nqblk = (((nqv + 31) >> 5) + 1) & ~1;  // query blocks, run in pairs

  // packed queries -> LDS: piece c (16 B) of query j at 16-B slot pk_slot(j, c) = j*8 + (c ^ ((j >> 1) & 7))
  // (conflict-free ds_read_b128 for a lane per query: any 16-lane group of the read covers all 16
  // columns of 16 B); thresholds
  for (int p = threadIdx.x; p < SQPB * 8; p += SNW * 64) {
    const int j = p >> 3, c = p & 7, q = qbase + j;
    const bool qok = q < nq && (!rerun || rerun[q]);
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (qok) v = reinterpret_cast<const uint4*>(queries + (int64_t)q * 128)[c];
    reinterpret_cast<uint4*>(qpk)[pk_slot(j, c)] = v;
  }
  for (int j = threadIdx.x; j < SQPB; j += SNW * 64) {
    const int q = qbase + j;
    const bool qok = q < nq && (!rerun || rerun[q]);
    int pc = 0;
    if (qok) {
      const uint4* qp = reinterpret_cast<const uint4*>(queries + (int64_t)q * 128);
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint4 v = qp[c];
        pc += __popc(v.x) + __popc(v.y) + __popc(v.z) + __popc(v.w);
      }
    }
    // dist < tau(q)  <=>  acc > 1024 + (pc(q) - tau(q)) / 2; padded and settled queries never accept
    thr[j] = qok ? 1024.0f + 0.5f * (float)(pc - tau[q]) : 1e30f;
    lcnt[j] = 0;
  }

  // LDS-DMA of row set rs into this wave's staging: SRS / 8 pieces of 64 x 16 B; 16-B slot i*64 + l holds
  // piece c of row r = 8i + (l >> 3) with pk_slot(r, c) = i*64 + l, i.e. c = (l & 7) ^ ((r >> 1) & 7),
  // where (r >> 1) & 7 = (4 (i & 1) + (l >> 4)) & 7: one column per parity of i.  Rows past the chunk
  // are clamped to its last row (their seeds mask them).
  const int dcol0 = ((l & 7) ^ ((l >> 4) & 7)) * 16, dcol1 = ((l & 7) ^ ((4 + (l >> 4)) & 7)) * 16;
  const int dlane0 = (l >> 3) * 128 + dcol0, dlane1 = (l >> 3) * 128 + dcol1;
  auto issue = [&](int rs) __attribute__((always_inline)) {
    const int64_t r0 = row0 + (int64_t)rs * SRS;
    if (r0 + SRS <= row1) {
      const uint8_t* base = codes + r0 * 128;
#pragma unroll
      for (int i = 0; i < SRS / 8; ++i) {
        const uint8_t* src = base + i * 1024 + ((i & 1) ? dlane1 : dlane0);
        uint8_t* dst = rst + i * 1024;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < SRS / 8; ++i) {
        int64_t row = r0 + 8 * i + (l >> 3);
        row = row < row1 ? row : row1 - 1;
        const uint8_t* src = codes + row * 128 + ((i & 1) ? dcol1 : dcol0);
        uint8_t* dst = rst + i * 1024;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    }
  };
  if (w < nrs) issue(w);
  __syncthreads();  // queries, thresholds and list lengths visible

  const uint32_t q0 = lds_addr(qpk), rst0 = lds_addr(rst), thr0 = lds_addr(thr), lc0 = lds_addr(lcnt);
  const uint32_t stg0 = lds_addr(stg), sdw0 = lds_addr(sdw);
  const int64_t qstride = (int64_t)nchunks * capc;
  uint64_t* const cbase = cand + ((int64_t)qbase * nchunks + chunk) * capc;  // + ql * qstride + pos
  int nst = 0;          // staged entries (wave-uniform)
  int ovf_qb = 1 << 20;  // the first query block whose hits went past the stage's end (wave-uniform)
  // staged hits of one row set (first row base_row) -> lists.  The stage holds the hits of the set's
  // query blocks 0 .. nqblk-1 in block order, so entries past STG are hits of blocks ovf_qb and later:
  // only those blocks' lists are marked overflowed (exact rescan), not the workgroup's 512 queries'.
  auto flush = [&](int64_t base_row) __attribute__((always_inline)) {
    if (nst > STG) {
      for (int i = ovf_qb * 32 + l; i < nqblk * 32; i += 64) lds_add32(lc0 + (uint32_t)(i * 4), capc + 1);
      nst = STG;
      ovf_qb = 1 << 20;
    }
    for (int i0 = 0; i0 < nst; i0 += 64) {
      const int i = i0 + l;
      int e = 0, pos = 0;
      if (i < nst) lds_read32(e, stg0 + (uint32_t)(i * 4));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(e)::"memory");
      const int ql = (e >> SENT_Q_SHIFT) & (SQPB - 1);
      if (i < nst) lds_add_rtn32(pos, lc0 + (uint32_t)(ql * 4), 1);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pos)::"memory");
      if (i < nst && pos < capc)
        cbase[(int64_t)ql * qstride + pos] =
            ((uint64_t)(uint32_t)(e >> SENT_V_SHIFT) << KEY_ROW_BITS) | (uint64_t)(base_row + (e & 127));
    }
    nst = 0;
  };
  // hits of row block rb against query block qbp (acc > th, th this lane's query threshold)
  auto block_hits = [&](const v16f& a, int rb, float th, int qbp) __attribute__((always_inline)) {
    uint32_t m16 = 0;
#pragma unroll
    for (int g = 0; g < 16; ++g) m16 |= (a[g] > th ? 1u : 0u) << g;
    int lo = l;  // lane-dependent values of this rare path from an opaque lane id (no hoisting)
    asm volatile("" : "+v"(lo));
    const int qrow = ((qbp * 32 + (lo & 31)) << SENT_Q_SHIFT) + 32 * rb + 4 * (lo >> 5);
    if (__ballot((m16 & (m16 - 1)) != 0)) {  // some lane holds two or more hits (rare): one ballot per register
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const uint64_t mask = __ballot((m16 >> g) & 1);
        if (mask) {
          if ((m16 >> g) & 1) {
            const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
            const int v = (int)(2.0f * th - 2.0f * a[g]);  // dist - tau(q) in [-1025, -1]
            const int pos = nst + below < STG ? nst + below : STG;
            lds_write32(stg0 + (uint32_t)(pos * 4), ((v + ENT_V_BIAS) << SENT_V_SHIFT) | (qrow + (g & 3) + 8 * (g >> 2)));
          }
          nst += __popcll(mask);
          if (nst > STG && qbp < ovf_qb) ovf_qb = qbp;
        }
      }
    } else {  // at most one hit per lane: it is the lane's largest register
      const uint64_t lanes = __ballot(m16 != 0);
      if (m16) {
        const v16i x = __builtin_bit_cast(v16i, a);
        const int x0 = max(max(x[0], x[1]), x[2]), x1 = max(max(x[3], x[4]), x[5]), x2 = max(max(x[6], x[7]), x[8]);
        const int x3 = max(max(x[9], x[10]), x[11]), x4 = max(max(x[12], x[13]), x[14]);
        const float mx = __int_as_float(max(max(max(x0, x1), x2), max(max(x3, x4), x[15])));
        const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(lanes >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)lanes, 0));
        const int g = __builtin_ctz(m16);
        const int v = (int)(2.0f * th - 2.0f * mx);
        const int pos = nst + below < STG ? nst + below : STG;
        lds_write32(stg0 + (uint32_t)(pos * 4), ((v + ENT_V_BIAS) << SENT_V_SHIFT) | (qrow + (g & 3) + 8 * (g >> 2)));
      }
      nst += __popcll(lanes);
      if (nst > STG && qbp < ovf_qb) ovf_qb = qbp;
    }
  };

  const int nmine = w < nrs ? (nrs - w + SNW - 1) / SNW : 0;  // this wave's row sets
  if (nmine > 0) {
    v4i A[SRB][KS];  // [rb][s]: dword 16h + s of row 32rb + ri of the row set, as 32 e2m1 values
    // seed of block row ri of row block rb at sdw[rb][hh][g], ri = (g & 3) + 8 (g >> 2) + 4 hh (lane halves
    // read 16 floats each); pc = the row's popcount, r = its row in the set
    auto write_seed = [&](int rb, int pc, int64_t r0) __attribute__((always_inline)) {
      const float sv = r0 + 32 * rb + ri < row1 ? 1024.0f - 0.5f * (float)pc : -4096.0f;
      if (h == 0)
        lds_write32(sdw0 + (uint32_t)((rb * 32 + ((ri >> 2) & 1) * 16 + (ri & 3) + 4 * (ri >> 3)) * 4), __float_as_int(sv));
    };
    // the row set's A fragments and seeds from the staging buffer (its DMA landed)
    auto rebuild = [&](int64_t r0) __attribute__((always_inline)) {
      static_for<0, SRB>([&](auto RB) {
        constexpr int rb = decltype(RB)::value;
        const int r = 32 * rb + ri;
        v4i p[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) lds_read128(p[i], rst0 + (uint32_t)(pk_slot(r, 4 * h + i) * 16));
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3])::"memory");
        int pc = 0;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const uint32_t wd = (uint32_t)p[s >> 2][s & 3];
          pc += __popc(wd);
          A[rb][s] = unpack_query32(wd);
          asm volatile("" : "+a"(A[rb][s]));  // straight to the accumulator file
        }
        pc += __shfl_xor(pc, 32, 64);  // both halves of the row
        write_seed(rb, pc, r0);
      });
    };
    // this lane half's 16 seeds of row block rb, as four 16-B reads
    // (the four reads land in the accumulator registers themselves; the caller's wait names them)
    auto read_seed = [&](int rb) __attribute__((always_inline)) {
      v4i p[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) lds_read128(p[i], sdw0 + (uint32_t)(rb * 128 + h * 64 + i * 16));
      const v16i x = __builtin_shufflevector(__builtin_shufflevector(p[0], p[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                             __builtin_shufflevector(p[2], p[3], 0, 1, 2, 3, 4, 5, 6, 7), 0, 1, 2, 3,
                                             4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
      return __builtin_bit_cast(v16f, x);
    };
    // the same, retired at once (the end of a spread switch: no copy of a register before its read lands)
    auto read_seed_now = [&](int rb) __attribute__((always_inline)) {
      v4i p[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) lds_read128(p[i], sdw0 + (uint32_t)(rb * 128 + h * 64 + i * 16));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3])::"memory");
      const v16i x = __builtin_shufflevector(__builtin_shufflevector(p[0], p[1], 0, 1, 2, 3, 4, 5, 6, 7),
                                             __builtin_shufflevector(p[2], p[3], 0, 1, 2, 3, 4, 5, 6, 7), 0, 1, 2, 3,
                                             4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
      return __builtin_bit_cast(v16f, x);
    };
    // query block qbi's B dwords (k-steps 4i..4i+3 in wq[i]) and this lane's threshold
    auto read_qblock = [&](v4i (&wq)[4], int& thb, int qbi) __attribute__((always_inline)) {
      const int j = qbi * 32 + ri;
#pragma unroll
      for (int i = 0; i < 4; ++i) lds_read128_inplace(wq[i], q0 + (uint32_t)(pk_slot(j, 4 * h + i) * 16));
      lds_read32_inplace(thb, thr0 + (uint32_t)(j * 4));
    };

    v16f acc[2][SRB];
    v4i wq[2][4] = {};
    int thb[2] = {};
    // retire every LDS read, naming the registers of parity c (accumulator seeds, B dwords, threshold)
    auto retire = [&](auto C) __attribute__((always_inline)) {
      constexpr int c = decltype(C)::value;
      (void)acc, (void)wq, (void)thb;  // (odr-use outside the if constexpr: clang's implicit capture)
      if constexpr (SRB == 2)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(acc[c][0]), "+v"(acc[c][1]), "+v"(wq[c][0]), "+v"(wq[c][1]), "+v"(wq[c][2]),
                       "+v"(wq[c][3]), "+v"(thb[c])::"memory");
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(acc[c][0]), "+v"(acc[c][1]), "+v"(acc[c][2]), "+v"(acc[c][3]), "+v"(wq[c][0]),
                       "+v"(wq[c][1]), "+v"(wq[c][2]), "+v"(wq[c][3]), "+v"(thb[c])::"memory");
    };
    // spread switch (SPREAD): packed dwords 4i..4i+3 of the lane's half row of row block rb of the next row
    // set (k-step group i) land in sg[rb], read in place one k-step before their group starts
    auto stage_read = [&](v4i (&sg)[SRB], int grp) __attribute__((always_inline)) {
      static_for<0, SRB>([&](auto RB) {
        constexpr int rb = decltype(RB)::value;
        lds_read128_inplace(sg[rb], rst0 + (uint32_t)(pk_slot(32 * rb + ri, 4 * h + grp) * 16));
      });
    };
    auto retire_sg = [&](v4i (&sg)[SRB]) __attribute__((always_inline)) {
      static_assert(!SPREAD || SRB == 4, "the wait names four row blocks' staging registers");
      if constexpr (SPREAD)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(sg[0]), "+v"(sg[1]), "+v"(sg[2]), "+v"(sg[3])::"memory");
    };

    wait_vm<0>();
    rebuild(row0 + (int64_t)w * SRS);
    if (nmine > 1) issue(w + SNW);
    static_for<0, SRB>([&](auto RB) { acc[0][RB] = read_seed(RB); });
    read_qblock(wq[0], thb[0], 0);
    retire(std::integral_constant<int, 0>{});

    bool have_prev = false;      // an untested block in acc[1 - parity]
    int prev_qb = 0;             // its query block
    int kset = 0;                // this wave's current row set (its k-th)
    int64_t set_base = row0 + (int64_t)w * SRS;  // first row of the current row set
    int64_t stage_base = set_base;               // ... of the row set the staged hits belong to
    // one query block: k-step s runs SRB MFMAs on the unpacked dword s of wq[c]; in the shadow: the
    // previous block's test (s = 1), the stage flush (s = 2), the next block's seeds, B dwords and
    // threshold (s = 3), retired at the top of the next block.  SW (the last block of a row set with the
    // spread switch): after k-step s's MFMAs, k-step s's A fragments of the next row set (its staging
    // read one k-step before its group of four starts); the next set's seeds and the DMA of the set
    // after it at the end.
    auto qblock = [&](auto PAR, auto SWC, int qbi) __attribute__((always_inline)) {
      constexpr int c = decltype(PAR)::value;
      constexpr bool SW = decltype(SWC)::value;
      retire(std::integral_constant<int, c>{});  // this block's operands (a no-op before the first)
      v4i sg[SRB] = {};   // SW: the next row set's packed dwords of one k-step group (block-local)
      int spc[SRB] = {};  // SW: its rows' popcounts (this lane's half row)
      if constexpr (SW) {  // the next row set's DMA (issued a whole set ago) landed: group 0
        wait_vm<0>();
        stage_read(sg, 0);
      }
      static_for<0, KS>([&](auto S) {
        constexpr int s = decltype(S)::value;
        const v4i bq = unpack_row32((uint32_t)wq[c][s >> 2][s & 3]);
        static_for<0, SRB>([&](auto RB) {
          acc[c][RB] = mfma_fp4(A[RB][s], bq, acc[c][RB]);
          // (SW: pinned before the fence, so the MFMAs reading A[.][s] are issued before A[.][s] is replaced)
          if constexpr (SW) asm volatile("" : "+v"(acc[c][RB]));
        });
        if constexpr (SW) VRQ_SCHED_FENCE();
        if constexpr (SW) {
          if constexpr ((s & 3) == 0) retire_sg(sg);
          static_for<0, SRB>([&](auto RB) {
            constexpr int rb = decltype(RB)::value;
            const uint32_t wd = (uint32_t)sg[rb][s & 3];
            spc[rb] += __popc(wd);
            A[rb][s] = unpack_query32(wd);  // k-step s of this block has issued its MFMAs
            asm volatile("" : "+a"(A[rb][s]));
          });
          if constexpr ((s & 3) == 3 && s < KS - 1) stage_read(sg, (s >> 2) + 1);
        }
        if constexpr (s == 1) {
          if (have_prev) {
            const float th = __int_as_float(thb[c ^ 1]);
            uint64_t hm[SRB], any = 0;
            static_for<0, SRB>([&](auto RB) {
              const v16i x = __builtin_bit_cast(v16i, acc[c ^ 1][RB]);
              const int x0 = max(max(x[0], x[1]), x[2]), x1 = max(max(x[3], x[4]), x[5]);
              const int x2 = max(max(x[6], x[7]), x[8]), x3 = max(max(x[9], x[10]), x[11]);
              const int x4 = max(max(x[12], x[13]), x[14]);
              hm[RB] = __ballot(max(max(max(x0, x1), x2), max(max(x3, x4), x[15])) > thb[c ^ 1]);
              any |= hm[RB];
            });
            if (any) {
              static_for<0, SRB>([&](auto RB) {
                if (hm[RB]) block_hits(acc[c ^ 1][RB], RB, th, prev_qb);
              });
            }
          }
        }
        if constexpr (s == 2) {
          // the first block of a set: every staged hit is the previous row set's
          if (qbi == 0) {
            if (have_prev && nst) flush(stage_base);
            stage_base = set_base;
          }
        }
        if constexpr (s == 3) {
          const int nxt = qbi + 1 < nqblk ? qbi + 1 : 0;
          if constexpr (!SW) static_for<0, SRB>([&](auto RB) { acc[c ^ 1][RB] = read_seed(RB); });  // (re-read after a switch)
          read_qblock(wq[c ^ 1], thb[c ^ 1], nxt);
        }
      });
      if constexpr (SW) {  // the next row set's seeds (its A fragments are in place), its successor's DMA
        const int64_t nb0 = row0 + (int64_t)(w + SNW * (kset + 1)) * SRS;
        static_for<0, SRB>([&](auto RB) {
          constexpr int rb = decltype(RB)::value;
          const int pc = spc[rb] + __shfl_xor(spc[rb], 32, 64);
          write_seed(rb, pc, nb0);
        });
        static_for<0, SRB>([&](auto RB) { acc[c ^ 1][RB] = read_seed_now(RB); });
        if (kset + 2 < nmine) issue(w + SNW * (kset + 2));  // (every staging read retired at k-step 12)
        set_base = nb0;
        ++kset;
      }
      have_prev = true;
      prev_qb = qbi;
    };

    using F = std::false_type;
    using T = std::true_type;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    // (SPREAD: the last pair of every row set switches, the last set's too -- it then rebuilds from a
    // stale staging buffer and nothing uses the result -- so that the loop body has one path and the
    // A fragments one register assignment)
    for (int k = 0; k < nmine; ++k) {
      if constexpr (SPREAD) {
        for (int qp = 0; qp + 2 < nqblk; qp += 2) {
          qblock(P0{}, F{}, qp);
          qblock(P1{}, F{}, qp + 1);
        }
        qblock(P0{}, F{}, nqblk - 2);
        qblock(P1{}, T{}, nqblk - 1);
      } else {  // (one copy of the pair in the loop body: the <2, 8> instance's code size and registers)
        for (int qp = 0; qp < nqblk; qp += 2) {
          qblock(P0{}, F{}, qp);
          qblock(P1{}, F{}, qp + 1);
        }
      }
      if (!SPREAD && k + 1 < nmine) {  // switch to the next row set: its DMA landed; start the one after
        wait_vm<0>();
        retire(P0{});
        set_base = row0 + (int64_t)(w + SNW * (k + 1)) * SRS;
        rebuild(set_base);
        if (k + 2 < nmine) issue(w + SNW * (k + 2));
        static_for<0, SRB>([&](auto RB) { acc[0][RB] = read_seed(RB); });
        retire(P0{});
      }
    }
    // the last block of the last row set
    {
      retire(P0{});
      const float th = __int_as_float(thb[1]);
      static_for<0, SRB>([&](auto RB) {
        const v16i x = __builtin_bit_cast(v16i, acc[1][RB]);
        const int x0 = max(max(x[0], x[1]), x[2]), x1 = max(max(x[3], x[4]), x[5]);
        const int x2 = max(max(x[6], x[7]), x[8]), x3 = max(max(x[9], x[10]), x[11]);
        const int x4 = max(max(x[12], x[13]), x[14]);
        if (__ballot(max(max(max(x0, x1), x2), max(max(x3, x4), x[15])) > thb[1])) block_hits(acc[1][RB], RB, th, prev_qb);
      });
      if (nst) flush(stage_base);
    }
  }
  wait_lgkm0();
  __syncthreads();  // every wave's list appends done
  for (int j = threadIdx.x; j < SQPB; j += SNW * 64) {
    const int q = qbase + j;
    if (q < nq && (!rerun || rerun[q])) ccnt[(int64_t)q * nchunks + chunk] = lcnt[j];
  }
}

// ---------------------------------------------------------------------------------------------
// K1r: the matrix-core scan for SMALL batches (nq <= 128): every wave streams its own rows.
//
// With few queries a row tile feeds few MFMAs, so sharing the unpacked tile between the four
// waves of a workgroup (K1m) does not pay for its barrier and LDS traffic: here each wave owns a
// contiguous chunk of rows, LDS-DMAs its own packed tiles (ring of NPR per wave, no barrier), and
// unpacks each 32-bit piece of a row straight into the B fragment registers of one k-step.  All MB
// M-blocks (32 queries each, MB*32 >= nq) of the batch are in every wave.
//   k-step s, lane (ri, h): dword 16h + s of row ri (so a lane reads its 64 contiguous bytes of
//   the row: 4 conflict-free ds_read_b128 through the tile swizzle), queries the same dword.
// Same thresholds (sampled tau_s / exact re-run with tau_p), same per-(query, chunk) lists and
// suffix merge as K1m; the hit path flushes synchronously (hits are rare at the sizes this serves).
// MB = 1 runs two workgroups per CU (two waves per SIMD at <= 256 VGPR + AGPR, a ring of 2 tiles per
// wave), so one wave's MFMAs run while the other waits on its tile or unpacks; MB = 2 / 4 need more
// than 256 registers and keep one wave per SIMD with a ring of 3 tiles.
//
// Registers an LDS read (inline asm: the compiler cannot see when it lands) writes are never copied
// before the wait that retires it: the packed rows of the next n-block go to the register set of
// the other parity (rb[par ^ 1], consumed in place by the next n-block, no cur = nxt copy the
// register allocator could hoist above the wait), and every such register is an operand of that
// wait.  (Round 4: a v_mov of in-flight rows placed before the s_waitcnt gave wrong distances on
// ~1 in 10^4 candidates; tests/test_capi.py::test_no_copies_of_inflight_lds_reads checks the ISA.)
template <int MB>
struct RowsShape {
  static_assert(MB == 1 || MB == 4, "M-blocks per wave (MB = 2: hamming_mfma_rows_lean_kernel)");
  static constexpr int QPW = 32 * MB;
  static constexpr int OCC = MB == 1 ? 2 : 1;  // workgroups (of MWAVES single-wave chunks) per CU
  static constexpr int NPR = MB == 1 ? 2 : 3;  // packed ring depth per wave (tile t+NPR-1 in flight)
  static constexpr bool SEEDREG = MB <= 2;     // accumulator seeds kept in registers (else re-read from LDS)
  static constexpr int SMEM = MWAVES * (NPR * PKT + QPW * 8 + (STG + 1) * 4 + MB * 128);
  static_assert(SMEM * OCC <= 160 * 1024, "LDS budget");
};
constexpr int K1R_AUX = 2;  // cache policy of the row DMA: nt (each row is read by one wave once per batch)

template <int MODE, int MB>
__global__ __launch_bounds__(MWAVES * 64, RowsShape<MB>::OCC) void hamming_mfma_rows_kernel(
    const uint8_t* __restrict__ codes, int64_t n, const uint8_t* __restrict__ queries, int nq,
    const int32_t* __restrict__ tau, uint64_t* __restrict__ cand, int32_t* __restrict__ ccnt, int capc,
    int64_t chunk_rows, int64_t chunk_stride, int64_t tile_stride, int nchunks, const int32_t* __restrict__ rerun,
    const int32_t* __restrict__ qbflag, uint16_t* __restrict__ dv, int64_t dv_stride) {
  // DENSE = the sample pass (as K1m's): chunk c = this wave's T tiles, tile t at row
  // c * chunk_stride + t * tile_stride (every tile whole), lane minima to dv[q][c * 32 + lane row]
  constexpr bool DENSE = MODE == MFMA_SAMPLE;
  constexpr int QPW = RowsShape<MB>::QPW;
  constexpr int NPR = RowsShape<MB>::NPR;
  constexpr bool SEEDREG = RowsShape<MB>::SEEDREG;
  if (qbflag && qbflag[0] == 0) return;  // re-run pass with no failed query
  __shared__ __attribute__((aligned(16))) uint8_t smem[RowsShape<MB>::SMEM];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* pk = smem + w * (NPR * PKT);  // this wave's ring
  int32_t* wbase = reinterpret_cast<int32_t*>(smem + MWAVES * NPR * PKT);
  int32_t* lcnt = wbase + w * QPW;                      // this wave's list lengths
  int32_t* tq = wbase + MWAVES * QPW + w * QPW;         // tau'(q) = tau(q) - pc(q)
  int32_t* stg = wbase + 2 * MWAVES * QPW + w * (STG + 1);  // hit staging (+1 spare)
  float* sd = reinterpret_cast<float*>(wbase + 2 * MWAVES * QPW + MWAVES * (STG + 1)) + w * MB * 32;
  const int l = lane_id();
  const int h = l >> 5, ri = l & 31;
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, q8 = nb >> 3, r8 = nb & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int chunk = L * MWAVES + w;
  if (chunk >= nchunks) return;
  const int64_t row0 = (int64_t)chunk * chunk_stride;
  const bool strided = tile_stride != RT;
  const int64_t row1 = strided ? n : (row0 + chunk_rows < n) ? row0 + chunk_rows : n;
  if (row0 >= row1) return;
  const int nrows = strided ? (int)chunk_rows : (int)(row1 - row0);
  const int ntiles = (nrows + RT - 1) / RT;
  const int nblk = 2 * ntiles;  // 32-row n-blocks

  // LDS-DMA of packed tile t: 8 pieces of 64 x 16 B (the K1m swizzle), the last partial tile clamped
  // to the chunk's last row.  (Source and destination of the builtin through locals: a compound
  // expression in its arguments makes the host-side compile silently drop the kernel's launch stub.)
  uint32_t doff[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = i * 64 + l;
    const int r = p >> 3, c = (p & 7) ^ ((r >> 1) & 7);
    doff[i] = (uint32_t)(r * 128 + c * 16);
  }
  auto issue = [&](int t) __attribute__((always_inline)) {
    uint8_t* buf = pk + (t % NPR) * PKT;
    const int64_t tr0 = row0 + (int64_t)t * tile_stride;
    if (tr0 + RT <= row1) {
      const uint8_t* base = codes + tr0 * 128;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint8_t* src = base + doff[i];
        uint8_t* dst = buf + i * 1024;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, K1R_AUX);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        int64_t row = tr0 + (doff[i] >> 7);
        row = row < row1 ? row : row1 - 1;
        const uint8_t* src = codes + row * 128 + (doff[i] & 127);
        uint8_t* dst = buf + i * 1024;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
      }
    }
  };
  for (int t = 0; t < NPR && t < ntiles; ++t) issue(t);

  // A fragments: k-step s, lane (ri, h) = dword 16h + s of query 32m + ri
  v4i A[MB][KS];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int q = 32 * m + ri;
    const bool qok = q < nq && (!rerun || rerun[q]);
    const uint32_t* qp = reinterpret_cast<const uint32_t*>(queries + (int64_t)(qok ? q : 0) * 128);
    int pc = 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint32_t wd = qok ? qp[16 * h + s] : 0u;
      pc += __popc(wd);
      A[m][s] = unpack_query32(wd);
    }
    pc += __shfl_xor(pc, 32, 64);  // both halves of the query
    if (h == 0) tq[q] = DENSE ? 0 : qok ? tau[q] - pc : -0x40000000;
  }
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+a"(A[m][s]));
  for (int i = l; i < QPW; i += 64) lcnt[i] = 0;
#pragma unroll
  for (int m = 0; m < MB; ++m)
    if (l < 32) {
      const int g = l & 15, hh = l >> 4;
      sd[m * 32 + l] = 0.5f * (float)tq[32 * m + (g & 3) + 8 * (g >> 2) + 4 * hh];
    }
  const uint32_t sd0 = lds_addr(sd) + (uint32_t)(h * 64), stg0 = lds_addr(stg);
  const uint32_t lc0 = lds_addr(lcnt), pk0 = lds_addr(pk);
  // the accumulator seeds tau'/2 of M-block m: this lane's 16 values.  SYNC: retired here, before
  // the four pieces are joined; otherwise retired by the caller's wait, which names `a`
  auto load_seed = [&](v16f& a, int m, auto SYNC) __attribute__((always_inline)) {
    v4i p0, p1, p2, p3;
    lds_read128(p0, sd0 + (uint32_t)(m * 128));
    lds_read128(p1, sd0 + (uint32_t)(m * 128 + 16));
    lds_read128(p2, sd0 + (uint32_t)(m * 128 + 32));
    lds_read128(p3, sd0 + (uint32_t)(m * 128 + 48));
    if constexpr (decltype(SYNC)::value)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)::"memory");
    const v16i x = __builtin_shufflevector(__builtin_shufflevector(p0, p1, 0, 1, 2, 3, 4, 5, 6, 7),
                                           __builtin_shufflevector(p2, p3, 0, 1, 2, 3, 4, 5, 6, 7), 0, 1, 2, 3, 4,
                                           5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    a = __builtin_bit_cast(v16f, x);
  };
  // SEEDREG: the seeds stay in registers for the whole kernel and every n-block's first MFMA takes
  // them as its C operand; otherwise (MB = 4) they are re-read from LDS into the accumulators of
  // the other parity while this n-block's MFMAs run
  v16f seedv[SEEDREG ? MB : 1];
  v16f acc[2][MB];
  if constexpr (!DENSE) {
#pragma unroll
    for (int m = 0; m < MB; ++m) load_seed(SEEDREG ? seedv[SEEDREG ? m : 0] : acc[0][m], m, std::true_type{});
  }
  // this lane's 64 bytes of row (32 * (blk & 1) + ri) of the packed tile of n-block blk
  auto read_rows = [&](v4i (&d)[4], int blk) __attribute__((always_inline)) {
    const int r = 32 * (blk & 1) + ri;
    const uint32_t base = pk0 + (uint32_t)(((blk >> 1) % NPR) * PKT);
#pragma unroll
    for (int i = 0; i < 4; ++i) lds_read128(d[i], base + (uint32_t)(pk_slot(r, 4 * h + i) * 16));
  };
  // at most k tiles' DMA still in flight
  auto wait_tiles = [&](int k) __attribute__((always_inline)) {
    if (k <= 0) wait_vm<0>();
    else if (k == 1) wait_vm<8>();
    else wait_vm<16>();
  };
  static_assert(NPR - 1 <= 2, "wait_tiles covers up to 2 tiles in flight");
  wait_tiles((ntiles < NPR ? ntiles : NPR) - 1);  // tile 0 landed
  v4i rb[2][4];                                   // packed rows of the n-blocks of parity 0 / 1
  read_rows(rb[0], 0);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rb[0][0]), "+v"(rb[0][1]), "+v"(rb[0][2]), "+v"(rb[0][3])::"memory");

  const int64_t qstride = (int64_t)nchunks * capc;
  uint64_t* const cbase = cand + (int64_t)chunk * capc;  // + q * qstride + pos
  int nst = 0;
  auto flush_all = [&](int64_t base_row) __attribute__((always_inline)) {  // staged hits -> lists (sync)
    if (nst > STG) {
      for (int i = l; i < QPW; i += 64) lds_add32(lc0 + (uint32_t)(i * 4), capc + 1);
      nst = STG;
    }
    for (int i0 = 0; i0 < nst; i0 += 64) {
      const int i = i0 + l;
      int e = 0, pos = 0;
      if (i < nst) lds_read32(e, stg0 + (uint32_t)(i * 4));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(e)::"memory");
      const int ql = (e >> ENT_Q_SHIFT) & 127;
      if (i < nst) lds_add_rtn32(pos, lc0 + (uint32_t)(ql * 4), 1);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pos)::"memory");
      if (i < nst && pos < capc)
        cbase[(int64_t)ql * qstride + pos] =
            ((uint64_t)(uint32_t)(e >> ENT_V_SHIFT) << KEY_ROW_BITS) | (uint64_t)(base_row + (e & 127));
    }
    nst = 0;
  };
  auto block_hits = [&](const v16f& a, int m, int pc, float hp) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const uint64_t mask = __ballot(a[g] > hp);
      if (mask) {
        if ((mask >> l) & 1) {
          const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
          int lo = l;
          asm volatile("" : "+v"(lo));
          const int ql = 32 * m + (g & 3) + 8 * (g >> 2) + 4 * (lo >> 5);
          const int v = pc - (int)(2.0f * a[g]);  // dist - tau(q), as in K1m
          const int pos = nst + below < STG ? nst + below : STG;
          lds_write32(stg0 + (uint32_t)(pos * 4), ((v + ENT_V_BIAS) << ENT_V_SHIFT) | (ql << ENT_Q_SHIFT) | (lo & 31));
        }
        nst += __popcll(mask);
      }
    }
  };

  // DENSE: the 16 values v = dist - pc(q) of M-block m of an n-block (local row lr of the chunk) fold
  // into this lane's running minima (as K1m's)
  DenseMin<DENSE, MB> dmin;
  // ---- main loop over n-blocks; k-step s runs the MB MFMAs of n-block blk on the unpacked dword
  // s of rb[par], while the previous n-block's epilogue, this block's row popcount and the next
  // block's packed reads (into rb[par ^ 1]) fill the MFMA gaps ----
  int pcs = 0;       // running row popcount of this n-block (this lane's half)
  int pprev = 0;     // the previous n-block's row popcount (whole row)
  int hpb = 0x7fffffff;
  uint64_t hitm[MB];  // per M-block: lanes of the previous n-block with a candidate (wave-uniform)
#pragma unroll
  for (int m = 0; m < MB; ++m) hitm[m] = 0;
  auto nblock = [&](auto PAR, int blk) __attribute__((always_inline)) {
    constexpr int par = decltype(PAR)::value;  // blk & 1 (n-blocks run in pairs: static register sets)
    // the next n-block's tile: its DMA landed (tile boundary)
    if (par == 1 && blk + 1 < nblk) {
      const int t1 = (blk + 1) >> 1;  // tile about to be read
      const int last = t1 + NPR - 1 < ntiles ? t1 + NPR - 1 : ntiles - 1;  // last tile issued so far
      wait_tiles(last - t1);
    }
    const int lr = blk * 32 + ri;
    static_for<0, KS>([&](auto S) {
      constexpr int s = decltype(S)::value;
      const uint32_t wd = (uint32_t)rb[par][s >> 2][s & 3];
      const v4i bfrag = unpack_row32(wd);
      static_for<0, MB>([&](auto M) {
        constexpr int m = decltype(M)::value;
        if constexpr (s == 0 && DENSE)
          acc[par][m] = mfma_fp4(A[m][s], bfrag, v16f{});
        else if constexpr (s == 0 && SEEDREG)
          acc[par][m] = mfma_fp4(A[m][s], bfrag, seedv[SEEDREG ? m : 0]);
        else
          acc[par][m] = mfma_fp4(A[m][s], bfrag, acc[par][m]);
        asm volatile("" : "+v"(acc[par][m]));
      });
      VRQ_SCHED_FENCE();
      if constexpr (s == 0)
        pcs = __popc(wd);
      else
        pcs += __popc(wd);
      // epilogue of the previous n-block: tests (s = 1 .. MB), branch (s = MB + 1), re-seeds
      if constexpr (DENSE && s >= 1 && s < 1 + MB) {
        if (blk > 0) dmin.fold(acc[par ^ 1][s - 1], s - 1, pprev, lr - 32 < nrows);
      }
      if constexpr (!DENSE && s >= 1 && s < 1 + MB) {
        constexpr int m = s - 1;
        const v16i bb = __builtin_bit_cast(v16i, acc[par ^ 1][m]);
        const int x0 = max(max(bb[0], bb[1]), bb[2]), x1 = max(max(bb[3], bb[4]), bb[5]);
        const int x2 = max(max(bb[6], bb[7]), bb[8]), x3 = max(max(bb[9], bb[10]), bb[11]);
        const int x4 = max(max(bb[12], bb[13]), bb[14]);
        hitm[m] = __ballot(max(max(max(x0, x1), x2), max(max(x3, x4), bb[15])) > hpb);
      }
      if constexpr (!DENSE && s == MB + 1) {
        uint64_t any = hitm[0];  // (every hitm[m] assigned by this n-block's tests)
#pragma unroll
        for (int m = 1; m < MB; ++m) any |= hitm[m];
        if (any) {  // rare
          const int lrp = lr - 32;
          const int pc = lrp < nrows && blk > 0 ? pprev : 0x40000000;
          const float hp = 0.5f * (float)pc;
          static_for<0, MB>([&](auto M) {
            constexpr int mm = decltype(M)::value;
            if (hitm[mm]) block_hits(acc[par ^ 1][mm], mm, pc, hp);
          });
          if (nst) flush_all(row0 + (int64_t)(blk - 1) * 32);
        }
      }
      if constexpr (!DENSE && !SEEDREG && s >= MB + 2 && s < 2 * MB + 2)
        load_seed(acc[par ^ 1][s - MB - 2], s - MB - 2, std::false_type{});
      // the next n-block's packed data
      if constexpr (s == 8)
        if (blk + 1 < nblk) read_rows(rb[par ^ 1], blk + 1);
      VRQ_SCHED_FENCE();
    });
    // row popcount of this n-block (both halves) and its threshold for the next n-block's tests
    pprev = pcs + __shfl_xor(pcs, 32, 64);
    hpb = __float_as_int(0.5f * (float)(lr < nrows ? pprev : 0x40000000));
    // retire the reads of this n-block: every destination register is an operand of the wait
    if constexpr (!DENSE && !SEEDREG) {
      static_assert(MB == 4, "re-seeded instance");
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(rb[par ^ 1][0]), "+v"(rb[par ^ 1][1]), "+v"(rb[par ^ 1][2]), "+v"(rb[par ^ 1][3]),
                     "+v"(acc[par ^ 1][0]), "+v"(acc[par ^ 1][1]), "+v"(acc[par ^ 1][2]), "+v"(acc[par ^ 1][3])::"memory");
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(rb[par ^ 1][0]), "+v"(rb[par ^ 1][1]), "+v"(rb[par ^ 1][2]), "+v"(rb[par ^ 1][3])::"memory");
    }
    // tile t = blk >> 1 consumed once its second n-block's rows are in registers (rb[1], read during
    // the first n-block and retired here): refill its ring slot with the DMA of tile t + NPR
    if (par == 0 && (blk >> 1) + NPR < ntiles) issue((blk >> 1) + NPR);
  };
  for (int blk = 0; blk < nblk; blk += 2) {  // nblk is even
    nblock(std::integral_constant<int, 0>{}, blk);
    nblock(std::integral_constant<int, 1>{}, blk + 1);
  }
  // epilogue of the last n-block (odd parity)
  {
    constexpr int par = 1;
    const int lr = (nblk - 1) * 32 + ri;
    if constexpr (DENSE) {
      static_for<0, MB>([&](auto M) { dmin.fold(acc[par][decltype(M)::value], decltype(M)::value, pprev, lr < nrows); });
    } else {
      const int pc = lr < nrows ? pprev : 0x40000000;
      const float hp = 0.5f * (float)pc;
      static_for<0, MB>([&](auto M) {
        constexpr int mm = decltype(M)::value;
        if (any_above(acc[par][mm], hp)) block_hits(acc[par][mm], mm, pc, hp);
      });
      if (nst) flush_all(row0 + (int64_t)(nblk - 1) * 32);
    }
  }
  wait_lgkm0();
  if constexpr (DENSE)
    dmin.out(dv, dv_stride, (int64_t)chunk * 32 + ri, 0, h, nq);
  else
    for (int i = l; i < QPW; i += 64)
      if (i < nq && (!rerun || rerun[i])) ccnt[(int64_t)i * nchunks + chunk] = lcnt[i];
}

// K1r for batches of <= 64 queries (MB <= 2): the per-wave chunk scan of hamming_mfma_rows_kernel with
// a register budget that keeps TWO waves on every SIMD at MB = 2 as well (round 4; the MB = 2
// instance above holds 328 registers and runs one wave per SIMD, 0.58 of HBM at nq = 64):
//   * one accumulator set per M-block: the n-block's tests run after its 16 k-steps (the first test
//     waits for the last MFMA; the SIMD's other wave fills that gap) instead of in the next
//     n-block's MFMA shadow, which needed a second set;
//   * one set of packed-row registers: quad i (k-steps 4i .. 4i+3) of the NEXT n-block is read into
//     rb[i] right after k-step 4i+3 consumed it; all four are retired by one wait after the n-block's
//     tests (the last quad has had the tests' time to land), so no read is in flight across the loop
//     back-edge, where the register allocator may copy a loop-carried value;
//   * the seeds tau'/2 stay in registers (the C operand of every n-block's first MFMA).
// A, the thresholds, the lists and the DMA ring are as in hamming_mfma_rows_kernel (ring of 2 tiles
// per wave; tile t's slot is refilled once the last quad read from it has been retired).
template <int MB>
struct LeanShape {
  static_assert(MB == 2, "lean K1r: the MB = 2 instance");
  static constexpr int QPW = 32 * MB;
  static constexpr int OCC = 2;  // workgroups per CU (two waves per SIMD); mfma_plan sizes the chunks by it
  static constexpr int NPR = 2;
  static constexpr int SMEM = MWAVES * (NPR * PKT + QPW * 8 + (STG + 1) * 4 + MB * 128);
  static_assert(OCC * SMEM <= 160 * 1024, "LDS budget of two workgroups per CU");
};

template <int MODE, int MB>
__global__ __launch_bounds__(MWAVES * 64, LeanShape<MB>::OCC) void hamming_mfma_rows_lean_kernel(
    const uint8_t* __restrict__ codes, int64_t n, const uint8_t* __restrict__ queries, int nq,
    const int32_t* __restrict__ tau, uint64_t* __restrict__ cand, int32_t* __restrict__ ccnt, int capc,
    int64_t chunk_rows, int64_t chunk_stride, int64_t tile_stride, int nchunks, const int32_t* __restrict__ rerun,
    const int32_t* __restrict__ qbflag, uint16_t* __restrict__ dv, int64_t dv_stride) {
  constexpr bool DENSE = MODE == MFMA_SAMPLE;
  constexpr int QPW = LeanShape<MB>::QPW, NPR = LeanShape<MB>::NPR;
  if (qbflag && qbflag[0] == 0) return;  // re-run pass with no failed query
  __shared__ __attribute__((aligned(16))) uint8_t smem[LeanShape<MB>::SMEM];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* pk = smem + w * (NPR * PKT);  // this wave's ring
  int32_t* wbase = reinterpret_cast<int32_t*>(smem + MWAVES * NPR * PKT);
  int32_t* lcnt = wbase + w * QPW;
  int32_t* tq = wbase + MWAVES * QPW + w * QPW;
  int32_t* stg = wbase + 2 * MWAVES * QPW + w * (STG + 1);
  float* sd = reinterpret_cast<float*>(wbase + 2 * MWAVES * QPW + MWAVES * (STG + 1)) + w * MB * 32;
  const int l = lane_id();
  const int h = l >> 5, ri = l & 31;
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, q8 = nb >> 3, r8 = nb & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int chunk = L * MWAVES + w;
  if (chunk >= nchunks) return;
  const int64_t row0 = (int64_t)chunk * chunk_stride;
  const bool strided = tile_stride != RT;
  const int64_t row1 = strided ? n : (row0 + chunk_rows < n) ? row0 + chunk_rows : n;
  if (row0 >= row1) return;
  const int nrows = strided ? (int)chunk_rows : (int)(row1 - row0);
  const int ntiles = (nrows + RT - 1) / RT;
  const int nblk = 2 * ntiles;

  // LDS-DMA of packed tile t: piece i (rows 8i .. 8i+7) of the K1m swizzle puts lane l at tile byte
  // i * 1024 + lo[i & 1] with lo[0] = (l >> 3) * 128 + ((l & 7) ^ (l >> 4)) * 16, lo[1] = lo[0] ^ 64:
  // two per-lane offsets (the byte offset of piece i is uniform), recomputed from an opaque lane id
  // at every issue so that no per-piece 64-bit address stays live across the loop
  auto issue = [&](int t) __attribute__((always_inline)) {
    int lo_ = l;
    asm volatile("" : "+v"(lo_));
    const uint32_t lo0 = (uint32_t)((lo_ >> 3) * 128 + ((lo_ & 7) ^ (lo_ >> 4)) * 16);
    uint8_t* buf = pk + (t % NPR) * PKT;
    const int64_t tr0 = row0 + (int64_t)t * tile_stride;
    const bool whole = tr0 + RT <= row1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t off = lo0 ^ (uint32_t)((i & 1) * 64);
      int64_t row = tr0 + 8 * i + (int64_t)(off >> 7);
      if (!whole) row = row < row1 ? row : row1 - 1;  // the last partial tile: clamp to the chunk's last row
      const uint8_t* src = codes + row * 128 + (off & 127);
      uint8_t* dst = buf + i * 1024;
      if (whole)
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, K1R_AUX);
      else
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  for (int t = 0; t < NPR && t < ntiles; ++t) issue(t);

  v4i A[MB][KS];
#pragma unroll
  for (int m = 0; m < MB; ++m) {
    const int q = 32 * m + ri;
    const bool qok = q < nq && (!rerun || rerun[q]);
    const uint32_t* qp = reinterpret_cast<const uint32_t*>(queries + (int64_t)(qok ? q : 0) * 128);
    int pc = 0;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const uint32_t wd = qok ? qp[16 * h + s] : 0u;
      pc += __popc(wd);
      A[m][s] = unpack_query32(wd);
    }
    pc += __shfl_xor(pc, 32, 64);
    if (h == 0) tq[q] = DENSE ? 0 : qok ? tau[q] - pc : -0x40000000;
  }
#pragma unroll
  for (int m = 0; m < MB; ++m)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+a"(A[m][s]));
  for (int i = l; i < QPW; i += 64) lcnt[i] = 0;
#pragma unroll
  for (int m = 0; m < MB; ++m)
    if (l < 32) {
      const int g = l & 15, hh = l >> 4;
      sd[m * 32 + l] = 0.5f * (float)tq[32 * m + (g & 3) + 8 * (g >> 2) + 4 * hh];
    }
  const uint32_t sd0 = lds_addr(sd) + (uint32_t)(h * 64), stg0 = lds_addr(stg);
  const uint32_t lc0 = lds_addr(lcnt), pk0 = lds_addr(pk);
  v16f seedv[MB];
  if constexpr (!DENSE) {
#pragma unroll
    for (int m = 0; m < MB; ++m) {
      v4i p0, p1, p2, p3;
      lds_read128(p0, sd0 + (uint32_t)(m * 128));
      lds_read128(p1, sd0 + (uint32_t)(m * 128 + 16));
      lds_read128(p2, sd0 + (uint32_t)(m * 128 + 32));
      lds_read128(p3, sd0 + (uint32_t)(m * 128 + 48));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3)::"memory");
      const v16i x = __builtin_shufflevector(__builtin_shufflevector(p0, p1, 0, 1, 2, 3, 4, 5, 6, 7),
                                             __builtin_shufflevector(p2, p3, 0, 1, 2, 3, 4, 5, 6, 7), 0, 1, 2, 3,
                                             4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
      seedv[m] = __builtin_bit_cast(v16f, x);
    }
  }
  // quad i of this lane's 64 bytes of row (32 * (blk & 1) + ri) of n-block blk's packed tile
  auto read_quad = [&](v4i& d, int i, int blk) __attribute__((always_inline)) {
    const int r = 32 * (blk & 1) + ri;
    lds_read128_inplace(d, pk0 + (uint32_t)(((blk >> 1) % NPR) * PKT) + (uint32_t)(pk_slot(r, 4 * h + i) * 16));
  };
  auto wait_tiles = [&](int k) __attribute__((always_inline)) {
    if (k <= 0) wait_vm<0>();
    else wait_vm<8>();
  };
  static_assert(NPR - 1 <= 1, "wait_tiles covers one tile in flight");
  wait_tiles((ntiles < NPR ? ntiles : NPR) - 1);  // tile 0 landed
  v4i rb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) read_quad(rb[i], i, 0);
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rb[0]), "+v"(rb[1]), "+v"(rb[2]), "+v"(rb[3])::"memory");

  const int64_t qstride = (int64_t)nchunks * capc;
  uint64_t* const cbase = cand + (int64_t)chunk * capc;
  int nst = 0;
  auto flush_all = [&](int64_t base_row) __attribute__((always_inline)) {
    if (nst > STG) {
      for (int i = l; i < QPW; i += 64) lds_add32(lc0 + (uint32_t)(i * 4), capc + 1);
      nst = STG;
    }
    for (int i0 = 0; i0 < nst; i0 += 64) {
      const int i = i0 + l;
      int e = 0, pos = 0;
      if (i < nst) lds_read32(e, stg0 + (uint32_t)(i * 4));
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(e)::"memory");
      const int ql = (e >> ENT_Q_SHIFT) & 127;
      if (i < nst) lds_add_rtn32(pos, lc0 + (uint32_t)(ql * 4), 1);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pos)::"memory");
      if (i < nst && pos < capc)
        cbase[(int64_t)ql * qstride + pos] =
            ((uint64_t)(uint32_t)(e >> ENT_V_SHIFT) << KEY_ROW_BITS) | (uint64_t)(base_row + (e & 127));
    }
    nst = 0;
  };
  auto block_hits = [&](const v16f& a, int m, int pc, float hp) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const uint64_t mask = __ballot(a[g] > hp);
      if (mask) {
        if ((mask >> l) & 1) {
          const int below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
          int lo = l;
          asm volatile("" : "+v"(lo));
          const int ql = 32 * m + (g & 3) + 8 * (g >> 2) + 4 * (lo >> 5);
          const int v = pc - (int)(2.0f * a[g]);
          const int pos = nst + below < STG ? nst + below : STG;
          lds_write32(stg0 + (uint32_t)(pos * 4), ((v + ENT_V_BIAS) << ENT_V_SHIFT) | (ql << ENT_Q_SHIFT) | (lo & 31));
        }
        nst += __popcll(mask);
      }
    }
  };
  DenseMin<DENSE, MB> dmin;
  v16f acc[MB];
  for (int blk = 0; blk < nblk; ++blk) {
    // entering the second n-block of tile t: the next n-block's quads (read from k-step 3 on) come from
    // tile t + 1, which must have landed (the wave's own DMA: no barrier)
    if ((blk & 1) && blk + 1 < nblk) {
      const int t1 = (blk + 1) >> 1;
      const int last = t1 + NPR - 1 < ntiles ? t1 + NPR - 1 : ntiles - 1;  // last tile issued so far
      wait_tiles(last - t1);
    }
    const int nx = blk + 1 < nblk ? blk + 1 : blk;
    int pcs = 0;
    static_for<0, KS>([&](auto S) {
      constexpr int s = decltype(S)::value;
      const uint32_t wd = (uint32_t)rb[s >> 2][s & 3];
#ifdef VRQ_K1R_PROBE_NOUNPACK  // timing-only probe builds (wrong results): the packed word as the B operand
      const v4i bfrag = {(int)wd, (int)wd, (int)wd, (int)wd};
#else
      const v4i bfrag = unpack_row32(wd);
#endif
      static_for<0, MB>([&](auto M) {
        constexpr int m = decltype(M)::value;
        if constexpr (s == 0 && DENSE)
          acc[m] = mfma_fp4(A[m][s], bfrag, v16f{});
        else if constexpr (s == 0)
          acc[m] = mfma_fp4(A[m][s], bfrag, seedv[m]);
        else
          acc[m] = mfma_fp4(A[m][s], bfrag, acc[m]);
        asm volatile("" : "+v"(acc[m]));
      });
      VRQ_SCHED_FENCE();
      pcs += __popc(wd);
      // (unconditional: the last n-block re-reads its own rows, unused -- a read under a branch would
      // merge two register sets at the join, by copies the allocator may place before the wait)
      if constexpr ((s & 3) == 3) read_quad(rb[s >> 2], s >> 2, nx);
      VRQ_SCHED_FENCE();
    });
    // epilogue of this n-block (its rows: local lr)
    const auto pp = __builtin_amdgcn_permlane32_swap((uint32_t)pcs, (uint32_t)pcs, false, false);
    const int prow = (int)(pp[0] + pp[1]);  // row popcount (both lane halves)
    const int lr = blk * 32 + ri;
    if constexpr (DENSE) {
      static_for<0, MB>([&](auto M) { dmin.fold(acc[decltype(M)::value], decltype(M)::value, prow, lr < nrows); });
    } else {
      const int pc = lr < nrows ? prow : 0x40000000;
      const float hp = 0.5f * (float)pc;
      const int hpb = __float_as_int(hp);
      uint64_t hitm[MB];
      uint64_t any = 0;
      static_for<0, MB>([&](auto M) {
        constexpr int m = decltype(M)::value;
        const v16i bb = __builtin_bit_cast(v16i, acc[m]);
        const int x0 = max(max(bb[0], bb[1]), bb[2]), x1 = max(max(bb[3], bb[4]), bb[5]);
        const int x2 = max(max(bb[6], bb[7]), bb[8]), x3 = max(max(bb[9], bb[10]), bb[11]);
        const int x4 = max(max(bb[12], bb[13]), bb[14]);
        hitm[m] = __ballot(max(max(max(x0, x1), x2), max(max(x3, x4), bb[15])) > hpb);
        any |= hitm[m];
      });
      if (any) {  // rare
        static_for<0, MB>([&](auto M) {
          constexpr int m = decltype(M)::value;
          if (hitm[m]) block_hits(acc[m], m, pc, hp);
        });
        if (nst) flush_all(row0 + (int64_t)blk * 32);
      }
    }
    // the next n-block's rows landed (every destination named)
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(rb[0]), "+v"(rb[1]), "+v"(rb[2]), "+v"(rb[3])::"memory");
    // after n-block 2t every read from tile t is retired: its ring slot takes the DMA of tile t + NPR
    // (issued before the wait for tile t + 1 at the top of n-block 2t+1, which counts it)
    if (!(blk & 1) && (blk >> 1) + NPR < ntiles) issue((blk >> 1) + NPR);
  }
  wait_lgkm0();
  if constexpr (DENSE)
    dmin.out(dv, dv_stride, (int64_t)chunk * 32 + ri, 0, h, nq);
  else
    for (int i = l; i < QPW; i += 64)
      if (i < nq && (!rerun || rerun[i])) ccnt[(int64_t)i * nchunks + chunk] = lcnt[i];
}

// Thresholds from the dense sample (S rows spread over the corpus, every distance exact):
//   tau_p(q) = d_(K) + 1, accept dist <= the K-th smallest sample distance: the sample rows alone
//              put >= K corpus rows under it, so the candidates always hold the exact top-K
//              (the guaranteed threshold of the re-run);
//   tau_s(q) = d_(j) + 1 for the plan's j < K: with iid rows the corpus holds ~j*n/S rows under
//              it, >= K with probability 1 - 1e-6 (plan); sample_check_kernel proves it per query.
// One workgroup per query: histogram of the S u16 values v + 1024 (v = dist - pc(q)).
__global__ __launch_bounds__(256) void sample_select_kernel(const uint16_t* __restrict__ dv, int64_t S,
                                                            const uint8_t* __restrict__ queries, int K, int j,
                                                            int32_t* __restrict__ tau_s, int32_t* __restrict__ tau_p,
                                                            int32_t* __restrict__ rerun, int32_t* __restrict__ qbflag,
                                                            int nqb) {
  constexpr int NB = 2049;
  __shared__ uint32_t hist[NB + 3];
  __shared__ int pcq;
  const int qi = blockIdx.x, tid = threadIdx.x;
  if (qi == 0 && qbflag)
    for (int i = tid; i < nqb; i += 256) qbflag[i] = 0;
  for (int i = tid; i < NB; i += 256) hist[i] = 0;
  if (tid == 0) pcq = 0;
  __syncthreads();
  if (tid < 32) atomicAdd(&pcq, __popc(reinterpret_cast<const uint32_t*>(queries + (int64_t)qi * 128)[tid]));
  const uint16_t* d = dv + (int64_t)qi * S;
  const int64_t S8 = S & ~int64_t(7);
  // 16-B loads of 8 values, 8 loads in flight per thread (one workgroup per query: with few queries
  // the pass is latency-bound on a handful of CUs)
  constexpr int U = 8;
  auto add8 = [&](const uint4& w) {
    const uint32_t x[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t lo = x[k] & 0xffff, hi = x[k] >> 16;
      if (lo < NB) atomicAdd(&hist[lo], 1u);
      if (hi < NB) atomicAdd(&hist[hi], 1u);
    }
  };
  int64_t i = (int64_t)tid * 8;
  for (; i + (U - 1) * 256 * 8 < S8; i += U * 256 * 8) {
    uint4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) w[u] = *reinterpret_cast<const uint4*>(d + i + u * 256 * 8);
#pragma unroll
    for (int u = 0; u < U; ++u) add8(w[u]);
  }
  for (; i < S8; i += 256 * 8) add8(*reinterpret_cast<const uint4*>(d + i));
  for (int64_t i = S8 + tid; i < S; i += 256)
    if (d[i] < NB) atomicAdd(&hist[d[i]], 1u);
  __syncthreads();
  if (tid < 64) {  // one wave: prefix sums over NB bins, 33 per lane
    constexpr int BPL = (NB + 63) / 64;
    int loc = 0;
    for (int i = 0; i < BPL; ++i) {
      const int b = tid * BPL + i;
      if (b < NB) loc += (int)hist[b];
    }
    int inc = loc;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if (tid >= o) inc += y;
    }
    // k-th smallest: bin b holds it iff cum < k <= cum + hist[b]
    int cum = inc - loc, rk = NB, rj = NB;
    for (int i = 0; i < BPL; ++i) {
      const int b = tid * BPL + i;
      if (b < NB) {
        const int hh = (int)hist[b];
        if (cum < K && cum + hh >= K) rk = b;
        if (cum < j && cum + hh >= j) rj = b;
        cum += hh;
      }
    }
    for (int o = 32; o > 0; o >>= 1) {
      rk = min(rk, __shfl_xor(rk, o, 64));
      rj = min(rj, __shfl_xor(rj, o, 64));
    }
    if (tid == 0) {
      // fewer than K valid sample values (not for a planned sample): accept every row
      const int dk = rk < NB ? rk - 1024 + pcq : 1024;
      const int dj = rj < NB ? rj - 1024 + pcq : 1024;
      tau_p[qi] = dk + 1;
      tau_s[qi] = (j < K ? dj : dk) + 1;
      rerun[qi] = 0;  // (the suffix reads tau_p for re-run queries; until a recheck, none)
    }
  }
}

// Proof of the sampled threshold per query: C = candidates with dist < tau_s over the whole corpus
// (the list lengths; an overflowed list counts > capc, and its exact rescan needs no threshold).
// C >= K means the K-th smallest key of the corpus has dist < tau_s, so the candidates hold the
// exact top-K.  Otherwise the query is flagged for the re-run with tau_p.  One wave per query.
__global__ __launch_bounds__(256) void sample_check_kernel(const int32_t* __restrict__ ccnt, int nchunks, int K,
                                                           int nq, int32_t* __restrict__ rerun,
                                                           int32_t* __restrict__ qbflag, int qpb) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), l = lane_id();
  if (q >= nq) return;
  int64_t c = 0;
  for (int i = l; i < nchunks; i += 64) c += ccnt[(int64_t)q * nchunks + i];
  c = wave_sum_i64(c);
  const bool fail = c < K;
  if (l == 0) {
    rerun[q] = fail ? 1 : 0;
    if (fail) atomicOr(&qbflag[q / qpb], 1);
  }
}

// Suffix candidates -> one sorted list of K keys per query (KEY_NONE padded).
// The matrix-core kernel left, per (query, chunk), a list of keys (v + 1025) << 40 | row
// (v = dist - tau(q)) and its length.  Exact in every case:
//   all lists complete, total <= SUF_CAP  -> sort them all;
//   all lists complete, total  > SUF_CAP  -> histogram of v, threshold T = K-th smallest v, sort
//                                            the keys with v <= T (if they fit);
//   some list overflowed (or neither fits) -> exact rescan of the query's suffix rows.
constexpr int SUF_THREADS = 256;
constexpr int SUF_CAP = 4096;
constexpr int SUF_COFF = 2049 + 3;  // chunk offsets of the parallel list gather live in the histogram's space
struct SufShared {
  uint32_t hist[2049 + 3];
  uint64_t buf[SUF_CAP];
  uint32_t qw[32];
  int32_t misc[8];
  int32_t scan[SUF_THREADS / WAVE];
};

__device__ __forceinline__ int row_dist(const uint8_t* __restrict__ codes, int64_t r, const uint32_t* qw) {
  const uint4* p = reinterpret_cast<const uint4*>(codes + r * 128);
  int d = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const uint4 v = p[c];
    d += __popc(v.x ^ qw[4 * c]) + __popc(v.y ^ qw[4 * c + 1]) + __popc(v.z ^ qw[4 * c + 2]) +
         __popc(v.w ^ qw[4 * c + 3]);
  }
  return d;
}

// block-wide exclusive scan (SUF_THREADS threads), total in *tot
__device__ inline int suf_excl_scan(int v, int* tot, int32_t* scratch) {
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
  for (int i = 0; i < SUF_THREADS / WAVE; ++i) {
    const int s = scratch[i];
    if (i < w) base += s;
    all += s;
  }
  __syncthreads();
  *tot = all;
  return base + x - v;
}

// Exact top-K of the query's suffix rows [row_begin, n) by brute force (one workgroup): distance
// histogram -> threshold T, then the dist < T rows (any order, sorted by the caller) and the
// first R rows with dist == T in row order.  Leaves m keys (real dist) in sh.buf; returns m.
__device__ int suffix_rescan(const uint8_t* __restrict__ codes, int64_t n, int64_t row_begin, int K, SufShared& sh) {
  const int tid = threadIdx.x;
  for (int i = tid; i < 1025; i += SUF_THREADS) sh.hist[i] = 0;
  __syncthreads();
  uint32_t qw[32];
  for (int i = 0; i < 32; ++i) qw[i] = sh.qw[i];
  for (int64_t r = row_begin + tid; r < n; r += SUF_THREADS) atomicAdd(&sh.hist[row_dist(codes, r, qw)], 1u);
  __syncthreads();
  if (tid == 0) {
    int cum = 0, T = 1025, clt = 0;
    for (int d = 0; d < 1025; ++d) {
      if (cum + (int)sh.hist[d] >= K) {
        T = d;
        clt = cum;
        break;
      }
      cum += (int)sh.hist[d];
    }
    if (T == 1025) clt = cum;
    sh.misc[0] = T;
    sh.misc[1] = clt;
    sh.misc[2] = 0;  // dist < T appended
    sh.misc[3] = 0;  // dist == T taken
  }
  __syncthreads();
  const int T = sh.misc[0], clt = sh.misc[1];
  const int R = K - clt;
  for (int64_t base = row_begin; base < n; base += SUF_THREADS) {
    const int64_t r = base + tid;
    const int d = r < n ? row_dist(codes, r, qw) : 0x7fffffff;
    if (d < T) {
      const int pos = atomicAdd(&sh.misc[2], 1);
      sh.buf[pos] = ((uint64_t)(uint32_t)d << KEY_ROW_BITS) | (uint64_t)r;
    }
    const int eq = (d == T) ? 1 : 0;
    if (__syncthreads_or(eq)) {
      int tot;
      const int pre = suf_excl_scan(eq, &tot, sh.scan);  // rank among this block's eq rows, row order
      const int rank = sh.misc[3] + pre;
      if (eq && rank < R) sh.buf[clt + rank] = ((uint64_t)(uint32_t)d << KEY_ROW_BITS) | (uint64_t)r;
      __syncthreads();
      if (tid == 0) sh.misc[3] += tot;
      __syncthreads();
    }
  }
  __syncthreads();
  const int taken = sh.misc[3] < R ? sh.misc[3] : R;
  return clt + (taken > 0 ? taken : 0);
}

__global__ __launch_bounds__(SUF_THREADS) void suffix_topk_kernel(const uint8_t* __restrict__ codes, int64_t n,
                                                                   int64_t row_begin,
                                                                   const uint8_t* __restrict__ queries,
                                                                   const uint64_t* __restrict__ cand,
                                                                   const int32_t* __restrict__ ccnt, int nchunks,
                                                                   int capc, int K, const int32_t* __restrict__ tau_main,
                                                                   const int32_t* __restrict__ tau_p,
                                                                   const int32_t* __restrict__ rerun,
                                                                   uint64_t* __restrict__ out) {
  __shared__ SufShared sh;
  const int qi = blockIdx.x, tid = threadIdx.x;
  if (tid < 32) sh.qw[tid] = reinterpret_cast<const uint32_t*>(queries + (int64_t)qi * 128)[tid];
  if (tid < 8) sh.misc[tid] = 0;
  __syncthreads();
  if (tid < 32) atomicAdd(&sh.misc[4], __popc(sh.qw[tid]));  // pc(q)
  const int32_t* cq = ccnt + (int64_t)qi * nchunks;
  const uint64_t* Cq = cand + (int64_t)qi * nchunks * capc;
  // per-chunk counts -> offsets (CPT chunks per thread)
  const int CPT = (nchunks + SUF_THREADS - 1) / SUF_THREADS;
  int mine = 0, over = 0;
  for (int j = 0; j < CPT; ++j) {
    const int c = tid * CPT + j;
    if (c < nchunks) {
      const int v = cq[c];
      over |= v > capc;
      mine += v < capc ? v : capc;
    }
  }
  int total;
  int off = suf_excl_scan(mine, &total, sh.scan);
  const bool overflow = __syncthreads_or(over) != 0;
  // the threshold the query's lists were recorded with: the main pass's, or tau_p after a re-run;
  // dist = v-field + tau(q) - ENT_V_BIAS
  const int tauq = (rerun && rerun[qi]) ? tau_p[qi] : tau_main[qi];
  const int64_t dfix = (int64_t)tauq - ENT_V_BIAS;
  int m = -1;
  bool real_dist = false;
  if (!overflow && total <= SUF_CAP && nchunks < SUF_COFF) {
    // every list entry gathered by its own thread (entry e of chunk c = the largest c with coff[c] <= e):
    // independent loads, all in flight at once (a per-thread loop over its chunks' entries waited for
    // each load before its LDS store)
    int32_t* coff = reinterpret_cast<int32_t*>(sh.hist);
    for (int j = 0; j < CPT; ++j) {
      const int c = tid * CPT + j;
      if (c < nchunks) {
        const int v = cq[c];
        coff[c] = off;
        off += v < capc ? v : capc;
      }
    }
    if (tid == 0) coff[nchunks] = total;
    __syncthreads();
    for (int e = tid; e < total; e += SUF_THREADS) {
      int lo = 0, hi = nchunks;  // coff[lo] <= e < coff[hi]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (coff[mid] <= e) lo = mid; else hi = mid;
      }
      sh.buf[e] = Cq[(int64_t)lo * capc + (e - coff[lo])];
    }
    m = total;
  } else if (!overflow && total <= SUF_CAP) {
    for (int j = 0; j < CPT; ++j) {
      const int c = tid * CPT + j;
      if (c < nchunks) {
        const int v = cq[c];
        for (int i = 0; i < v; ++i) sh.buf[off + i] = Cq[(int64_t)c * capc + i];
        off += v;
      }
    }
    m = total;
  } else if (!overflow) {
    // histogram over the v-field of every candidate, threshold T with >= K keys at v <= T
    for (int i = tid; i < 2049; i += SUF_THREADS) sh.hist[i] = 0;
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
      const int v = cq[c];
      for (int i = tid; i < v; i += SUF_THREADS)
        atomicAdd(&sh.hist[(uint32_t)(Cq[(int64_t)c * capc + i] >> KEY_ROW_BITS)], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      int cum = 0, T = 2048;
      for (int d = 0; d < 2049; ++d) {
        cum += (int)sh.hist[d];
        if (cum >= K) {
          T = d;
          break;
        }
      }
      sh.misc[5] = T;
      sh.misc[6] = cum;  // keys with v <= T
      sh.misc[7] = 0;
    }
    __syncthreads();
    if (sh.misc[6] <= SUF_CAP) {
      const uint32_t T = (uint32_t)sh.misc[5];
      for (int c = 0; c < nchunks; ++c) {
        const int v = cq[c];
        for (int i = tid; i < v; i += SUF_THREADS) {
          const uint64_t key = Cq[(int64_t)c * capc + i];
          if ((uint32_t)(key >> KEY_ROW_BITS) <= T) sh.buf[atomicAdd(&sh.misc[7], 1)] = key;
        }
      }
      __syncthreads();
      m = sh.misc[7];
    }
  }
  __syncthreads();
  if (m < 0) {  // overflowed list, or too many candidates: exact rescan (real distances)
    m = suffix_rescan(codes, n, row_begin, K, sh);
    real_dist = true;
  }
  __syncthreads();
  if (!real_dist && m > SUF_THREADS) {
    // only the keys with v <= T (T: the K-th smallest v-field) can be among the first K: histogram, then
    // keep those in place, so the sort below usually runs on ~K keys instead of every candidate
    for (int i = tid; i < 2049; i += SUF_THREADS) sh.hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < m; i += SUF_THREADS) atomicAdd(&sh.hist[(uint32_t)(sh.buf[i] >> KEY_ROW_BITS)], 1u);
    __syncthreads();
    {  // T = the smallest v with cum(v) >= K: BPT bins per thread, one block scan
      constexpr int BPT = (2049 + SUF_THREADS - 1) / SUF_THREADS;
      int loc = 0;
      for (int b = 0; b < BPT; ++b) {
        const int d = tid * BPT + b;
        if (d < 2049) loc += (int)sh.hist[d];
      }
      int tot;
      int cum = suf_excl_scan(loc, &tot, sh.scan);
      for (int b = 0; b < BPT; ++b) {
        const int d = tid * BPT + b;
        if (d >= 2049) break;
        const int h = (int)sh.hist[d];
        if (cum < K && cum + h >= K) sh.misc[5] = d;
        cum += h;
      }
      if (tid == 0) sh.misc[7] = 0;
    }
    __syncthreads();
    const uint32_t T = (uint32_t)sh.misc[5];
    constexpr int KPT = SUF_CAP / SUF_THREADS;  // keys per thread (m <= SUF_CAP)
    uint64_t kk[KPT];
#pragma unroll
    for (int j = 0; j < KPT; ++j) kk[j] = tid + j * SUF_THREADS < m ? sh.buf[tid + j * SUF_THREADS] : KEY_NONE;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < KPT; ++j)
      if (kk[j] != KEY_NONE && (uint32_t)(kk[j] >> KEY_ROW_BITS) <= T) sh.buf[atomicAdd(&sh.misc[7], 1)] = kk[j];
    __syncthreads();
    m = sh.misc[7];
  }
  if (m <= SUF_THREADS) {
    // one key per thread: its rank among the m distinct keys (broadcast LDS reads), one scatter
    const uint64_t ki = tid < m ? sh.buf[tid] : KEY_NONE;
    if (tid < 4) sh.buf[m + tid] = KEY_NONE;  // padding for the 4-key reads (m <= SUF_THREADS < SUF_CAP - 4)
    __syncthreads();
    int rank = 0;
    if (tid < m) {
      for (int j = 0; j < m; j += 4) {  // four broadcast reads in flight
        const uint64_t a = sh.buf[j], b = sh.buf[j + 1], c = sh.buf[j + 2], d = sh.buf[j + 3];
        rank += (a < ki ? 1 : 0) + (b < ki ? 1 : 0) + (c < ki ? 1 : 0) + (d < ki ? 1 : 0);
      }
    }
    __syncthreads();
    if (tid < m) sh.buf[rank] = ki;
    __syncthreads();
  } else {
    const int np2 = next_pow2(m);
    for (int i = m + tid; i < np2; i += SUF_THREADS) sh.buf[i] = KEY_NONE;
    __syncthreads();
    block_bitonic_sort_u64(sh.buf, np2);
  }
  uint64_t* o = out + (int64_t)qi * K;
  const uint64_t ROWM = (1ull << KEY_ROW_BITS) - 1;
  for (int i = tid; i < K; i += SUF_THREADS) {
    uint64_t key = KEY_NONE;
    if (i < m) {
      key = sh.buf[i];
      if (!real_dist) key = ((uint64_t)((int64_t)(key >> KEY_ROW_BITS) + dfix) << KEY_ROW_BITS) | (key & ROWM);
    }
    o[i] = key;
  }
}

// P(Poisson(lam) >= j) <= 1e-6: the sampled order j that an iid corpus proves with that probability
static int sample_order(double lam, int K) {
  double term = __builtin_exp(-lam), cdf = 0.0;
  for (int j = 1; j < K; ++j) {
    cdf += term;  // P(X <= j-1)
    if (1.0 - cdf <= 1e-6) return j;
    term *= lam / j;
  }
  return K;
}

int mfma_plan(int64_t n, int nq, int K, MfmaPlan* p) {
  if (nq < 1 || K < 1 || K > kMfmaMaxK) return VRQ_EUNSUPPORTED;
  // VRQ_MFMA_MB: probe-build override of the M-blocks per wave (2 or 4)
  const int em = tuning_int("VRQ_MFMA_MB", 0);
  p->mb = (em == 2 || em == 4) ? em : nq >= kMbLargeMinQueries ? kMbLarge : kMbSmall;
  p->qpb = p->mb == kMbLarge ? MfmaShape<kMbLarge>::QPB : MfmaShape<kMbSmall>::QPB;
  p->nqb = (nq + p->qpb - 1) / p->qpb;
  // large batches: K1s (row sets resident, queries streamed) for passes of <= kSwapMaxPairs (query, row)
  // pairs, K1m above (see kSwapMaxPairs)
  static_assert(SQPB == MfmaShape<kMbLarge>::QPB, "K1s serves K1m's MB = 4 query blocks");
  // (p->swap: 1 = K1s<2, 8>, 2 = K1s<4, 4>)
  {
    const bool short_pass = (double)n * (double)nq <= kSwapMaxPairs;
    p->swap = p->mb != kMbLarge ? 0 : short_pass ? (VRQ_K1S_RB4 ? 2 : 1) : (VRQ_K1S_LARGE ? 2 : 0);
  }
  // small batches (nq <= 128): the row-split kernel K1r, all queries in every wave
  // (VRQ_MFMA_ROWS=0: probe-build override)
  p->rows = nq <= kRowsMaxQueries && tuning_int("VRQ_MFMA_ROWS", 1) != 0;
  int rows_occ = 1;  // K1r workgroups per CU of the chosen instance
  if (p->rows) {
    p->swap = 0;
    p->mb = nq <= 32 ? 1 : nq <= 64 ? 2 : 4;
    p->qpb = kRowsMaxQueries;
    p->nqb = 1;
    rows_occ = p->mb == 1 ? RowsShape<1>::OCC : p->mb == 2 ? LeanShape<2>::OCC : RowsShape<4>::OCC;
  }
  // the dense sample pass always runs the MB = 2 instance (its 16 stores per block would spill at MB = 4)
  p->nqb_s = (nq + MfmaShape<kMbSmall>::QPB - 1) / MfmaShape<kMbSmall>::QPB;
  // sample: S rows in 64-row tiles spread evenly over the corpus at a tile stride ts >= 64 (a sample
  // robust to corpora stored in cluster order), in nsc chunks (one workgroup per CU and query block)
  // of T tiles: tile i = c*T + t starts at row i * ts, the last one inside [0, n).  S = n/32, at least
  // kMfmaMinSample and at most kMfmaMaxSample rows (the dense pass and its selection cost O(nq S)).
  // VRQ_SAMPLE_DIV: probe-build override of the sample fraction
  const int64_t ev = tuning_int("VRQ_SAMPLE_DIV", 0);
  const int64_t div = ev >= 2 ? ev : kMfmaSampleDiv;
  int64_t S = n / div;
  if (S > kMfmaMaxSample) S = kMfmaMaxSample;
  if (S < kMfmaMinSample) S = kMfmaMinSample;
  int64_t tiles = S / RT > 0 ? S / RT : 1;
  if (tiles > n / RT) tiles = n / RT;  // non-overlapping whole tiles (n >= kMfmaMinRows)
  // K1r with MB <= 2 runs the sample pass too (one sample chunk per wave); its MB = 4 instance would
  // spill in the dense epilogue, so batches of 65..128 queries take K1m's (MB = 2) sample pass
  p->rows_sample = p->rows && p->mb <= 2;
  int64_t nsc = p->rows_sample ? 256 * MWAVES * rows_occ : 256 / p->nqb_s;
  // >= 8 chunks: >= 256 lane minima per query (>= 2K; very large batches would otherwise keep
  // fewer than K values and fall back to accepting every row)
  if (nsc < 8) nsc = 8;
  if (nsc > tiles) nsc = tiles;
  const int64_t T = tiles / nsc;
  tiles = nsc * T;
  const int64_t ts = tiles > 1 ? (n - RT) / (tiles - 1) : RT;  // >= RT since (tiles - 1) * RT <= n - RT
  p->sample_chunk_rows = T * RT;
  p->sample_chunks = (int)nsc;
  p->sample_stride = T * ts;
  p->sample_tile_stride = ts;
  p->sample = tiles * RT;
  p->dvcols = nsc * 32;  // the dense pass writes 32 lane minima per (query, sample chunk)
  S = p->sample;
  // thresholded pass over all n rows (K1r: one chunk per wave, MWAVES waves per workgroup slot of a CU)
  int64_t want = p->rows ? 256 * MWAVES * rows_occ : 256 / p->nqb;
  if (want < 1) want = 1;
  int64_t cr = (n + want - 1) / want;
  cr = (cr + RT - 1) / RT * RT;
  if (cr < RT) cr = RT;
  p->chunk_rows = cr;
  p->nchunks = (int)((n + cr - 1) / cr);
  // per-(query, chunk) list capacity: 4x the hits expected under tau_p (K * cr / S, iid rows)
  const int64_t expect = (K * cr + S - 1) / S;
  int capc = 64;
  while (capc < 4 * expect && capc < 4096) capc <<= 1;
  p->capc = capc;
  p->j = sample_order((double)K * (double)S / (double)n, K);
  // workspace: dv [nq][dvcols] u16 | suffix list [nq][K] | cand [nq][nchunks][capc] |
  //            list lengths [nq][nchunks] | tau_s, tau_p, rerun [nq] | qbflag [nqb]
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  p->off_suffix = al((size_t)nq * p->dvcols * sizeof(uint16_t));
  p->off_cand = p->off_suffix + al((size_t)nq * K * sizeof(uint64_t));
  p->off_cnt = p->off_cand + al((size_t)nq * p->nchunks * p->capc * sizeof(uint64_t));
  p->off_tau = p->off_cnt + al((size_t)nq * p->nchunks * sizeof(int32_t));
  p->bytes = p->off_tau + 3 * al((size_t)nq * sizeof(int32_t)) + (size_t)p->nqb * sizeof(int32_t);
  return VRQ_OK;
}

bool mfma_use(int64_t n, int nq, int K, int flags) {
  if (flags & VRQ_SEARCH_SCAN_VALU) return false;
  const bool ok = K <= kMfmaMaxK && n >= kMfmaMinRows;
  if (flags & VRQ_SEARCH_SCAN_MFMA) return ok;
  return ok && nq >= kMfmaMinQueries;  // K1r serves even one query faster than the wavefront scan
}

int mfma_scan_launch(const MfmaPlan& p, const uint8_t* codes, int64_t n, const uint8_t* q, int nq, int K,
                     uint8_t* ws, hipStream_t s, int flags) {
  constexpr int ALL = VRQ_SCAN_STAGE_PREFIX | VRQ_SCAN_STAGE_MATRIX | VRQ_SCAN_STAGE_RECHECK | VRQ_SCAN_STAGE_SUFFIX;
  const int st = (flags & ALL) ? (flags & ALL) : ALL;
  uint16_t* dv = (uint16_t*)ws;
  uint64_t* suffix = (uint64_t*)(ws + p.off_suffix);
  uint64_t* cand = (uint64_t*)(ws + p.off_cand);
  int32_t* ccnt = (int32_t*)(ws + p.off_cnt);
  const size_t qa = ((size_t)nq * sizeof(int32_t) + 255) & ~size_t(255);
  int32_t* tau_s = (int32_t*)(ws + p.off_tau);
  int32_t* tau_p = (int32_t*)(ws + p.off_tau + qa);
  int32_t* rerun = (int32_t*)(ws + p.off_tau + 2 * qa);
  int32_t* qbflag = (int32_t*)(ws + p.off_tau + 3 * qa);
  const bool sampled = p.j < K;
  const int32_t* none = nullptr;
  // the MB = 4 or MB = 2 instance of a pass
  auto pass = [&](auto kswap2, auto kswap4, auto kern4, auto kern2, int grid, const int32_t* tau, uint64_t* cd,
                  int32_t* cc, int64_t crows, int64_t cstride, int nch, const int32_t* rr, const int32_t* qf,
                  uint16_t* d, int64_t dstride) {
    if (p.swap == 1)
      hipLaunchKernelGGL(kswap2, dim3(grid), dim3(8 * 64), 0, s, codes, n, (int64_t)0, q, nq, tau, cd, cc, p.capc,
                         crows, cstride, (int64_t)RT, nch, p.nqb, rr, qf, d, dstride);
    else if (p.swap == 2)
      hipLaunchKernelGGL(kswap4, dim3(grid), dim3(4 * 64), 0, s, codes, n, (int64_t)0, q, nq, tau, cd, cc, p.capc,
                         crows, cstride, (int64_t)RT, nch, p.nqb, rr, qf, d, dstride);
    else if (p.mb == kMbLarge)
      hipLaunchKernelGGL(kern4, dim3(grid), dim3(MWAVES * 64), 0, s, codes, n, (int64_t)0, q, nq, tau, cd, cc, p.capc,
                         crows, cstride, (int64_t)RT, nch, p.nqb, rr, qf, d, dstride);
    else
      hipLaunchKernelGGL(kern2, dim3(grid), dim3(MWAVES * 64), 0, s, codes, n, (int64_t)0, q, nq, tau, cd, cc, p.capc,
                         crows, cstride, (int64_t)RT, nch, p.nqb, rr, qf, d, dstride);
  };
  // K1r launches: the MB = 1 / 2 / 4 instance, one workgroup per MWAVES chunks
  auto rows_pass = [&](auto k1, auto k2, auto k4, const int32_t* tau, const int32_t* rr, const int32_t* qf,
                       int nch, int64_t crows, int64_t cstride, int64_t tstride, uint16_t* d, int64_t dstride) {
    const dim3 g((unsigned)((nch + MWAVES - 1) / MWAVES)), blk(MWAVES * 64);
    if (p.mb == 1)
      hipLaunchKernelGGL(k1, g, blk, 0, s, codes, n, q, nq, tau, cand, ccnt, p.capc, crows, cstride, tstride, nch, rr,
                         qf, d, dstride);
    else if (p.mb == 2)
      hipLaunchKernelGGL(k2, g, blk, 0, s, codes, n, q, nq, tau, cand, ccnt, p.capc, crows, cstride, tstride, nch, rr,
                         qf, d, dstride);
    else
      hipLaunchKernelGGL(k4, g, blk, 0, s, codes, n, q, nq, tau, cand, ccnt, p.capc, crows, cstride, tstride, nch, rr,
                         qf, d, dstride);
  };
  if ((st & VRQ_SCAN_STAGE_PREFIX) && p.rows_sample) {  // dense sample pass (K1r) + per-query thresholds
    // (rows_sample implies MB <= 2: the MB = 1 instance fills the unreachable MB = 4 slot)
    if (p.mb > 2) return VRQ_EUNSUPPORTED;
    rows_pass(hamming_mfma_rows_kernel<MFMA_SAMPLE, 1>, hamming_mfma_rows_lean_kernel<MFMA_SAMPLE, 2>,
              hamming_mfma_rows_kernel<MFMA_SAMPLE, 1>, none, none, none, p.sample_chunks, p.sample_chunk_rows,
              p.sample_stride, p.sample_tile_stride, dv, p.dvcols);
    VRQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(sample_select_kernel, dim3(nq), dim3(256), 0, s, (const uint16_t*)dv, p.dvcols, q, K, p.j,
                       tau_s, tau_p, rerun, qbflag, p.nqb);
    VRQ_LAUNCH_CHECK();
  } else if (st & VRQ_SCAN_STAGE_PREFIX) {  // dense sample pass + per-query thresholds
    hipLaunchKernelGGL((hamming_mfma_kernel<MFMA_SAMPLE, kMbSmall>), dim3(p.sample_chunks * p.nqb_s), dim3(MWAVES * 64),
                       0, s, codes, n, (int64_t)0, q, nq, none, (uint64_t*)nullptr, (int32_t*)nullptr, 0,
                       p.sample_chunk_rows, p.sample_stride, p.sample_tile_stride, p.sample_chunks, p.nqb_s, none,
                       none, dv, p.dvcols);
    VRQ_LAUNCH_CHECK();
    hipLaunchKernelGGL(sample_select_kernel, dim3(nq), dim3(256), 0, s, (const uint16_t*)dv, p.dvcols, q, K, p.j,
                       tau_s, tau_p, rerun, qbflag, p.nqb);
    VRQ_LAUNCH_CHECK();
  }
  if ((st & VRQ_SCAN_STAGE_MATRIX) && p.rows) {
    rows_pass(hamming_mfma_rows_kernel<MFMA_MAIN, 1>, hamming_mfma_rows_lean_kernel<MFMA_MAIN, 2>,
              hamming_mfma_rows_kernel<MFMA_MAIN, 4>, (const int32_t*)(sampled ? tau_s : tau_p), none, none,
              p.nchunks, p.chunk_rows, p.chunk_rows, (int64_t)RT, (uint16_t*)nullptr, (int64_t)0);
    VRQ_LAUNCH_CHECK();
  } else if (st & VRQ_SCAN_STAGE_MATRIX) {
#ifdef VRQ_K1M_STAMPS
    uint16_t* mdv = dv;
#else
    uint16_t* mdv = nullptr;
#endif
    pass(hamming_mfma_swap_kernel<MFMA_MAIN, 2, 8>, hamming_mfma_swap_kernel<MFMA_MAIN, 4, 4>,
         hamming_mfma_kernel<MFMA_MAIN, kMbLarge>,
         hamming_mfma_kernel<MFMA_MAIN, kMbSmall>, p.nchunks * p.nqb,
         (const int32_t*)(sampled ? tau_s : tau_p), cand, ccnt, p.chunk_rows, p.chunk_rows, p.nchunks, none, none,
         mdv, (int64_t)0);
    VRQ_LAUNCH_CHECK();
  }
  if ((st & VRQ_SCAN_STAGE_RECHECK) && sampled) {
    // prove C >= K per query; re-run the query blocks holding a failed query with tau_p
    hipLaunchKernelGGL(sample_check_kernel, dim3((nq + 3) / 4), dim3(256), 0, s, (const int32_t*)ccnt, p.nchunks, K,
                       nq, rerun, qbflag, p.qpb);
    VRQ_LAUNCH_CHECK();
    if (p.rows)
      rows_pass(hamming_mfma_rows_kernel<MFMA_RERUN, 1>, hamming_mfma_rows_lean_kernel<MFMA_RERUN, 2>,
                hamming_mfma_rows_kernel<MFMA_RERUN, 4>, (const int32_t*)tau_p, (const int32_t*)rerun,
                (const int32_t*)qbflag, p.nchunks, p.chunk_rows, p.chunk_rows, (int64_t)RT, (uint16_t*)nullptr,
                (int64_t)0);
    else
      pass(hamming_mfma_swap_kernel<MFMA_RERUN, 2, 8>, hamming_mfma_swap_kernel<MFMA_RERUN, 4, 4>,
           hamming_mfma_kernel<MFMA_RERUN, kMbLarge>,
           hamming_mfma_kernel<MFMA_RERUN, kMbSmall>, p.nchunks * p.nqb,
           (const int32_t*)tau_p, cand, ccnt, p.chunk_rows, p.chunk_rows, p.nchunks, (const int32_t*)rerun,
           (const int32_t*)qbflag, (uint16_t*)nullptr, (int64_t)0);
    VRQ_LAUNCH_CHECK();
  }
  if (st & VRQ_SCAN_STAGE_SUFFIX) {  // candidates of the whole corpus -> one sorted K-list per query
    hipLaunchKernelGGL(suffix_topk_kernel, dim3(nq), dim3(SUF_THREADS), 0, s, codes, n, (int64_t)0, q, cand, ccnt,
                       p.nchunks, p.capc, K, (const int32_t*)(sampled ? tau_s : tau_p), (const int32_t*)tau_p,
                       (const int32_t*)(sampled ? rerun : nullptr), suffix);
    VRQ_LAUNCH_CHECK();
  }
  return VRQ_OK;
}

}  // namespace vrq
