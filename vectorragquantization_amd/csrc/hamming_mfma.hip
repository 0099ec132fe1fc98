// hamming_mfma.hip -- K1m: Phase-I Hamming scan for LARGE query batches on the matrix cores.
//
// The wavefront popcount scan (hamming_scan.hip) costs 64 wave64 VALU instructions per
// (query, 1024-bit row) pair and a wave64 integer VALU op retires every 4 cycles
// (tools/probes/valu_probe.hip): beyond ~16 queries per pass it is VALU-bound.  Here the
// same distances come from v_mfma_i32_32x32x32_i8 on 0/1 bytes:
//     dist(q, r) = popcount(q) + popcount(r) - 2 * <bits(q), bits(r)>
// which is exact (integer accumulation), so Phase-I ranks stay bit-identical to FAISS.
//
// Work decomposition: one 256-thread workgroup per CU (LDS ~152 KiB), one wave per SIMD so
// each wave owns the full 512-entry register file:
//  * each wave holds the A fragments of 64 queries (2 M-blocks of 32) for the whole K = 1024
//    (256 registers, unpacked once) and their thresholds;
//  * 64-row tiles of PACKED codes stream HBM -> LDS by LDS-DMA (XOR-swizzled source, ring of
//    3); while the matrix core runs tile t, the same waves expand tile t+1 into int8 0/1
//    B fragments laid out [n-block][k-step][lane][16 B] (each MFMA operand read is one
//    contiguous ds_read_b128) and the rows' popcounts -- VALU work issued in the gaps between
//    MFMAs.  One barrier per tile hands the unpacked tile over (double buffer).
//  * Epilogue per tile: v = pcr - 2*acc compared against tau'(q) = tau(q) - pcq(q); a row is
//    a candidate iff dist < tau(q), where tau(q) is the exact K-th smallest distance of the
//    query over a PREFIX of the corpus (computed by the exact scan).  FAISS admits a row only
//    if dist < heap_top, rows in increasing index: a suffix row with dist >= tau(q) ranks
//    after >= K prefix rows, so the strict test loses nothing.  Candidates are appended to a
//    per-(query, chunk) list owned by one wave (ballot/mbcnt positions, no atomics);
//    suffix_topk_kernel merges them into one sorted K-list per query, exactly in every case.
#include "vrq_internal.h"
#include "vrq_scan.h"

// tools/probes/mfma_bisect.hip compiles this file with VRQ_BISECT bits set to time the kernel
// with parts removed (1: epilogue, 2: unpack, 4: MFMA).  Never set in the library build.
#ifndef VRQ_BISECT
#define VRQ_BISECT 0
#endif

namespace vrq {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

constexpr int MWAVES = 4;                   // waves per workgroup (one per SIMD)
constexpr int QPW = 64;                     // queries per wave
constexpr int QPB = MWAVES * QPW;           // queries per workgroup (256)
constexpr int RT = 64;                      // rows per tile (2 n-blocks of 32)
constexpr int KS = 16;                      // k-steps of 64 bits (1024-bit codes)
constexpr int PKT = RT * 128;               // packed tile bytes (8 KiB)
constexpr int NPK = 4;                      // packed ring depth (DMA issued 4 tiles ahead)
constexpr int NUB = 3;                      // unpacked ring: tile t read, t+1 ready, t+2 written
constexpr int UBT = 2 * KS * 1024;          // unpacked tile bytes (32 KiB)
constexpr int GPW = (PKT / 1024) / MWAVES;  // LDS-DMA instructions per wave per tile (2)
constexpr int STG = 448;                    // per-wave LDS staging of candidate hits
constexpr int SMEM_BYTES = NPK * PKT + NUB * UBT + NUB * RT * 4 + MWAVES * 64 * 4 + MWAVES * STG * 12;
constexpr int E8M0_TWO = 128;               // MX block scale 2^1
constexpr int FMT_FP4 = 4;                  // e2m1 operand format of the f8f6f4 MFMA

__device__ __forceinline__ void barrier_all() { asm volatile("s_barrier" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// 32 code bits -> one FP4 MFMA fragment lane: 32 e2m1 values, code 0x1 (0.5) per set bit.
// Dword j, nibble i holds bit 4i + j: a fixed permutation of k applied identically to queries
// (A) and rows (B), so every dot product is unchanged.  Two ops per dword.
__device__ __forceinline__ v8i unpack32(uint32_t bits) {
  v8i r = {0, 0, 0, 0, 0, 0, 0, 0};
  r[0] = (int)(bits & 0x11111111u);
  r[1] = (int)((bits >> 1) & 0x11111111u);
  r[2] = (int)((bits >> 2) & 0x11111111u);
  r[3] = (int)((bits >> 3) & 0x11111111u);
  return r;
}

// (0.5 * 2^1) * (0.5 * 2^1) = 1 per common set bit: C + popcount(q & r) exactly (<= 1024 in f32)
__device__ __forceinline__ v16f mfma_fp4(const v8i& a, const v8i& b, const v16f& c) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, FMT_FP4, FMT_FP4, 0, E8M0_TWO, 0, E8M0_TWO);
}

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
template <int OFF>
__device__ __forceinline__ void lds_read128o(v4i& d, uint32_t a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "i"(OFF) : "memory");
}
__device__ __forceinline__ void lds_read32(int& d, uint32_t a) {
  asm volatile("ds_read_b32 %0, %1" : "=v"(d) : "v"(a) : "memory");
}
__device__ __forceinline__ void lds_write128(uint32_t a, const v4i& v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_write64(uint32_t a, uint64_t v) {
  asm volatile("ds_write_b64 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_read64(uint64_t& d, uint32_t a) {
  asm volatile("ds_read_b64 %0, %1" : "=v"(d) : "v"(a) : "memory");
}
__device__ __forceinline__ void lds_write32(uint32_t a, int v) {
  asm volatile("ds_write_b32 %0, %1" ::"v"(a), "v"(v) : "memory");
}
#define VRQ_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

// Packed tile image: 16-byte piece c of tile row r lives at slot r*8 + (c ^ ((r>>1)&7)).
__device__ __forceinline__ int pk_slot(int r, int c) { return r * 8 + (c ^ ((r >> 1) & 7)); }

__global__ __launch_bounds__(MWAVES * 64, 1) void hamming_mfma_kernel(
    const uint8_t* __restrict__ codes, int64_t n, int64_t row_begin, const uint8_t* __restrict__ queries, int nq,
    const int32_t* __restrict__ tau, uint64_t* __restrict__ cand, int32_t* __restrict__ ccnt, int capc,
    int64_t chunk_rows, int nchunks, int nqb) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[SMEM_BYTES];
  uint8_t* pk = smem;                                       // NPK packed tiles
  uint8_t* ub = smem + NPK * PKT;                           // NUB unpacked tiles
  int32_t* pcr = (int32_t*)(smem + NPK * PKT + NUB * UBT);  // NUB x 64 row popcounts
  // tau(q) - pc(q) per wave, [m][h][g]: the query of accumulator register g in lane-half h
  int32_t* taul = pcr + NUB * RT + (threadIdx.x >> 6) * 64;
  // per-wave hit staging: STG keys (u64) then STG destination offsets (u32)
  uint8_t* stg = (uint8_t*)(pcr + NUB * RT + MWAVES * 64) + (threadIdx.x >> 6) * STG * 12;

  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l = lane_id();
  const int h = l >> 5, ri = l & 31;
  // XCD-aware bijective remap: consecutive logical blocks share one XCD's L2
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, q8 = nb >> 3, r8 = nb & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int chunk = L / nqb;
  const int qb = L - chunk * nqb;
  if (chunk >= nchunks) return;
  const int64_t row0 = row_begin + (int64_t)chunk * chunk_rows;
  const int64_t row1 = (row0 + chunk_rows < n) ? row0 + chunk_rows : n;
  const int nrows = (int)(row1 - row0);
  const int ntiles = (nrows + RT - 1) / RT;

  auto issue = [&](int t) {
    uint8_t* buf = pk + (t % NPK) * PKT;
    const int64_t tr0 = row0 + (int64_t)t * RT;
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const int gi = w * GPW + i;
      const int p = gi * 64 + l;  // LDS slot written by this lane
      const int r = p >> 3, cs = p & 7;
      const int c = cs ^ ((r >> 1) & 7);
      int64_t row = tr0 + r;
      row = row < row1 ? row : row1 - 1;
      __builtin_amdgcn_global_load_lds(codes + row * 128 + c * 16,
                                       (__attribute__((address_space(3))) void*)(buf + gi * 1024), 16, 0, 0);
    }
  };
  const uint32_t pk0 = lds_addr(pk), ub0 = lds_addr(ub), pcr0 = lds_addr(pcr);
  // unit u of this wave = (nblk, piece) = ((4w+u) >> 3, (4w+u) & 7): lane -> tile row
  // 32*nblk + ri; piece p (dwords 4p..4p+3) holds k-steps 2p, 2p+1; lane-half h takes dword
  // 2j+h of step 2p+j.
  uint32_t usrc[4], udst[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int unit = 4 * w + u, nblk = unit >> 3, p = unit & 7;
    const int r = nblk * 32 + ri;
    usrc[u] = (uint32_t)(pk_slot(r, p) * 16);
    udst[u] = (uint32_t)(((nblk * KS + 2 * p) * 64 + l) * 16);
  }
  // row popcounts: tile rows 16w..16w+15, 4 lanes per row, 2 pieces each
  const int pr = 16 * w + (l >> 2), pc0 = 2 * (l & 3);
  const uint32_t psrc0 = (uint32_t)(pk_slot(pr, pc0) * 16), psrc1 = (uint32_t)(pk_slot(pr, pc0 + 1) * 16);
  auto unpack_write = [&](const v4i& v, int u, uint32_t ubuf) {
    const v8i f0 = unpack32((uint32_t)(h ? v.y : v.x)), f1 = unpack32((uint32_t)(h ? v.w : v.z));
    lds_write128(ubuf + udst[u], (v4i){f0[0], f0[1], f0[2], f0[3]});
    lds_write128(ubuf + udst[u] + 1024, (v4i){f1[0], f1[1], f1[2], f1[3]});
  };
  auto rowpc_write = [&](const v4i& a, const v4i& c, uint32_t pbuf) {
    int pc = __popc(a.x) + __popc(a.y) + __popc(a.z) + __popc(a.w) + __popc(c.x) + __popc(c.y) + __popc(c.z) +
             __popc(c.w);
    pc += __builtin_amdgcn_update_dpp(0, pc, 0xB1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
    pc += __builtin_amdgcn_update_dpp(0, pc, 0x4E, 0xf, 0xf, false);  // quad_perm [2,3,0,1]
    if ((l & 3) == 0) lds_write32(pbuf + (uint32_t)(pr * 4), pc);
  };

  // ---- prologue: DMA tiles 0..3, A fragments + thresholds, unpack tiles 0 and 1 ----
  for (int t = 0; t < NPK && t < ntiles; ++t) issue(t);

  const int qbase = qb * QPB + w * QPW;
  v8i A[2][KS];  // [m][s]: bits 64s+32h .. +31 of query qbase + 32m + ri as 32 e2m1 values
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int q = qbase + 32 * m + ri;
    const bool qok = q < nq;
    const uint4* qp = reinterpret_cast<const uint4*>(queries + (int64_t)(qok ? q : 0) * 128);
    int pc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint4 v = qp[c];
      const uint32_t wd[4] = {qok ? v.x : 0u, qok ? v.y : 0u, qok ? v.z : 0u, qok ? v.w : 0u};
      pc += __popc(wd[0]) + __popc(wd[1]) + __popc(wd[2]) + __popc(wd[3]);
      A[m][2 * c] = unpack32(h ? wd[1] : wd[0]);
      A[m][2 * c + 1] = unpack32(h ? wd[3] : wd[2]);
    }
    // lane (ri, h=0) holds query ri's threshold; slot [m][h'][g] wants query (g&3)+8(g>>2)+4h'
    const int tl = qok ? tau[q] - pc : -0x40000000;  // padded queries never accept
    if (h == 0) {
      const int g = (ri & 3) | ((ri >> 3) << 2);     // inverse of (g&3) + 8(g>>2)
      taul[(m * 2 + ((ri >> 2) & 1)) * 16 + g] = tl;
    }
  }
  // A lives in the accumulator file (MFMA reads it from there), freeing the VGPRs for the B ring
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+a"(A[m][s]));
  __syncthreads();
  // accumulator seed tau'/2 per register: after the K loop acc = <q,r> + tau'/2, and the row is
  // a candidate iff pc(r) - 2<q,r> < tau'  <=>  acc > pc(r)/2
  v16f seed[2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int g = 0; g < 16; ++g) seed[m][g] = 0.5f * (float)taul[(m * 2 + h) * 16 + g];

  if (ntiles >= 4)
    wait_vm<2 * GPW>();
  else if (ntiles == 3)
    wait_vm<GPW>();
  else
    wait_vm<0>();
  barrier_all();  // packed tiles 0 and 1 visible to all waves
  {
    v4i pv[8], pa[2], pb[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int u = 0; u < 4; ++u) lds_read128(pv[4 * t + u], pk0 + (uint32_t)(t * PKT) + usrc[u]);
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
  if (ntiles >= 4)
    wait_vm<GPW>();
  else
    wait_vm<0>();
  wait_lgkm0();

  // ---- epilogue helpers: block (m, nbk) of a finished tile ----
  // accumulator register g = query (g&3)+8(g>>2)+4h of M-block m, tile row 32*nbk + ri.
  // A hit stores key (v + 1024) << 40 | row with v = pc(row) - 2<q,row> = dist - pc(q) (the
  // same order as dist for a fixed query).
  auto block_any = [&](const v16f& a, float half_pc) -> uint64_t {
    float mx = fmaxf(fmaxf(a[0], a[1]), a[2]);
    mx = fmaxf(fmaxf(mx, a[3]), a[4]);
    mx = fmaxf(fmaxf(mx, a[5]), a[6]);
    mx = fmaxf(fmaxf(mx, a[7]), a[8]);
    mx = fmaxf(fmaxf(mx, a[9]), a[10]);
    mx = fmaxf(fmaxf(mx, a[11]), a[12]);
    mx = fmaxf(fmaxf(mx, a[13]), a[14]);
    mx = fmaxf(mx, a[15]);
    return __ballot(mx > half_pc);
  };
  // list lengths in registers: lcr[m][g] of lane-half h = list of query (g&3)+8(g>>2)+4h of
  // M-block m (uniform per half); stride between consecutive queries' lists in cand
  int lcr[2][16];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int g = 0; g < 16; ++g) lcr[m][g] = 0;
  const int64_t qstride = (int64_t)nchunks * capc;
  // this wave's lists: query qbase + ql, chunk `chunk` -> cbase + ql * qstride + pos
  uint64_t* const cbase = cand + ((int64_t)qbase * nchunks + chunk) * capc;
  // Hits are staged in LDS and written to HBM after the end-of-tile DMA wait: a global store
  // issued between a tile's DMA and that wait would make vmcnt wait for the DMA just issued.
  const uint32_t stk0 = lds_addr(stg), sto0 = stk0 + STG * 8;
  int nst = 0;  // staged entries (wave-uniform)
  auto flush = [&]() {
    for (int i0 = 0; i0 < nst; i0 += 64) {
      const int i = i0 + l;
      uint64_t key = 0;
      int off = -1;
      if (i < nst) {
        lds_read64(key, stk0 + (uint32_t)(i * 8));
        lds_read32(off, sto0 + (uint32_t)(i * 4));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(key), "+v"(off)::"memory");
      if (i < nst && off >= 0) cbase[off] = key;
    }
    nst = 0;
  };
  // hits of registers g0..g0+7 of a block (the any-test already found one in the block)
  auto block_hits = [&](const v16f& a, int m, int g0, int pc, float half_pc, int64_t row) {
    const uint64_t rowbits = (uint64_t)row;
#pragma unroll
    for (int g = g0; g < g0 + 8; ++g) {
      const bool hit = a[g] > half_pc;
      const uint64_t mask = __ballot(hit);
      if (mask) {
        const uint32_t lo = (uint32_t)mask, hi = (uint32_t)(mask >> 32);
        const int below = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0));
        const int pos = lcr[m][g] + (h ? below - __popc(lo) : below);
        const int cnt = __popc(lo) + __popc(hi);
        if (nst + cnt <= STG) {
          if (hit) {
            const int v = pc - 2 * (int)(a[g] - seed[m][g]);  // exact integers
            const int ql = 32 * m + (g & 3) + 8 * (g >> 2) + 4 * h;
            lds_write64(stk0 + (uint32_t)((nst + below) * 8),
                        ((uint64_t)(uint32_t)(v + 1024) << KEY_ROW_BITS) | rowbits);
            lds_write32(sto0 + (uint32_t)((nst + below) * 4), pos < capc ? (int)(ql * qstride + pos) : -1);
          }
          lcr[m][g] += __popc(h ? hi : lo);
          nst += cnt;
        } else {
          // staging full (> STG hits in one tile): mark the list overflowed; the suffix step
          // rescans this query exactly
          lcr[m][g] = capc + 1;
        }
      }
    }
  };
  auto block_pc = [&](int pcv, int lr) { return lr < nrows ? pcv : 0x40000000; };  // past the end: no hit
  // ---- main loop: 16 regions of 4 chained MFMAs per tile ----
  // Region r computes k-steps 4(r&3)..+3 of block b = r>>2 = (m, nbk) = (b>>1, b&1) into
  // acc[b&1]; the B fragment of each MFMA is read 2 regions ahead into a 4-slot ring (across
  // the tile boundary: tile t+1 is complete before iteration t starts).  Unpack of tile t+2
  // (one unit per 4 regions) and the epilogue of the previous block run in the MFMA shadow.
  v4i ring[4][4];
  v16f acc[2];
  auto read_region = [&](int slot_, uint32_t ubuf, int r) {
    const int bb = r >> 2, qq = r & 3, nbk = bb & 1;
    const uint32_t base = ubuf + (uint32_t)(((nbk * KS + 4 * qq) * 64 + l) * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) lds_read128(ring[slot_][j], base + (uint32_t)(j * 1024));
  };
  int pcvP[2] = {0, 0};  // previous tile's row popcounts (block 3 = nbk 1)
  barrier_all();         // B_0: unpacked tiles 0 and 1, packed tile 2 visible
  read_region(0, ub0, 0);
  read_region(1, ub0, 1);
  for (int t = 0; t < ntiles; ++t) {
    if (t + 4 < ntiles) issue(t + 4);  // into the slot of tile t (unpacked in iteration t-2)
    const uint32_t ubt = ub0 + (uint32_t)((t % NUB) * UBT);
    const uint32_t ubn = ub0 + (uint32_t)(((t + 1) % NUB) * UBT);
    const uint32_t ubw = ub0 + (uint32_t)(((t + 2) % NUB) * UBT);
    const uint32_t pks = pk0 + (uint32_t)(((t + 2) % NPK) * PKT);
    int pcvN[2];
    lds_read32(pcvN[0], pcr0 + (uint32_t)(((t % NUB) * RT + ri) * 4));
    lds_read32(pcvN[1], pcr0 + (uint32_t)(((t % NUB) * RT + 32 + ri) * 4));
    v4i pv, pa, pb;
    uint64_t anyb = 0;
    VRQ_SCHED_FENCE();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int bk = r >> 2, qq = r & 3, m = bk >> 1;
      // B fragments of region r+2 (tile t+1 for r >= 14)
      if (r + 2 < 16)
        read_region((r + 2) & 3, ubt, r + 2);
      else
        read_region((r + 2) & 3, ubn, r + 2 - 16);
      // packed reads two regions before their use (regions 3, 7, 11, 15 unpack; 15 row pcs)
      if ((r & 3) == 1) lds_read128(pv, pks + usrc[r >> 2]);
      if (r == 13) {
        lds_read128(pa, pks + psrc0);
        lds_read128(pb, pks + psrc1);
      }
      // region r's fragments: >= 8 LDS ops were issued after them
      asm volatile("s_waitcnt lgkmcnt(8)"
                   : "+v"(ring[r & 3][0]), "+v"(ring[r & 3][1]), "+v"(ring[r & 3][2]), "+v"(ring[r & 3][3]),
                     "+v"(pv), "+v"(pcvN[0]), "+v"(pcvN[1])::"memory");
      v16f& c = acc[bk & 1];
#pragma unroll
      for (int j = 0; j < ((VRQ_BISECT & 4) ? 0 : 4); ++j) {
        const int s = 4 * qq + j;
        const v4i& bf = ring[r & 3][j];
        const v8i bv = {bf.x, bf.y, bf.z, bf.w, 0, 0, 0, 0};
        c = mfma_fp4(A[m][s], bv, s == 0 ? seed[m] : c);
      }
      if (VRQ_BISECT & 4) {
        if (qq == 0) c = seed[m];
      }
      // pin the accumulator here: the MFMA intrinsics are pure, and without a use at this point
      // IR-level sinking moves them past the scheduling fences
      asm volatile("" : "+a"(c));
      if ((r & 3) == 3 && !(VRQ_BISECT & 2)) unpack_write(pv, r >> 2, ubw);
      if (r == 15) {
        asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(pa), "+v"(pb)::"memory");
        if (!(VRQ_BISECT & 2)) rowpc_write(pa, pb, pcr0 + (uint32_t)(((t + 2) % NUB) * RT * 4));
      }
      // epilogue of the previous block pb (block 3 of tile t-1 in regions 1-3): any-test in
      // region 4bk+1, hits of registers 0-7 / 8-15 in regions 4bk+2 / 4bk+3
      if ((r & 3) >= 1 && !(VRQ_BISECT & 1)) {
        const bool prev_tile = bk == 0;
        const int pb_ = prev_tile ? 3 : bk - 1;
        if (!prev_tile || t > 0) {
          const v16f& pa_ = acc[pb_ & 1];
          const int mm = pb_ >> 1, nbk = pb_ & 1;
          const int lr = (prev_tile ? (t - 1) : t) * RT + nbk * 32 + ri;
          const int pc = block_pc(prev_tile ? pcvP[1] : pcvN[nbk], lr);
          const float hp = 0.5f * (float)pc;
          if ((r & 3) == 1)
            anyb = block_any(pa_, hp);
          else if (anyb)
            block_hits(pa_, mm, ((r & 3) - 2) * 8, pc, hp, row0 + lr);
        }
      }
      VRQ_SCHED_FENCE();
    }
    pcvP[0] = pcvN[0];
    pcvP[1] = pcvN[1];
    // packed tile t+3 (unpacked next iteration) landed; this wave's LDS writes done
    if (t + 4 < ntiles)
      wait_vm<GPW>();
    else
      wait_vm<0>();
    wait_lgkm0();
    if (nst) flush();  // this tile's hits -> HBM; they drain while the next tile runs
    barrier_all();     // B_{t+1}
  }
  if (ntiles > 0 && !(VRQ_BISECT & 1)) {  // block 3 of the last tile
    const int lr = (ntiles - 1) * RT + 32 + ri;
    const int pc = block_pc(pcvP[1], lr);
    const float hp = 0.5f * (float)pc;
    if (block_any(acc[1], hp)) {
      block_hits(acc[1], 1, 0, pc, hp, row0 + lr);
      block_hits(acc[1], 1, 8, pc, hp, row0 + lr);
    }
  }
  if (nst) flush();
  if (ri == 0) {  // lanes 0 and 32 hold their half's lengths
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int q = qbase + 32 * m + (g & 3) + 8 * (g >> 2) + 4 * h;
        if (q < nq) ccnt[(int64_t)q * nchunks + chunk] = lcr[m][g];
      }
  }
}

// Exact prefix threshold: tau(q) = K-th smallest distance over the union of the prefix
// chunk lists; 1025 (admit every suffix row) when the prefix holds fewer than K rows.
__global__ __launch_bounds__(256) void prefix_tau_kernel(const uint64_t* __restrict__ lists, int nl, int K,
                                                         int32_t* __restrict__ tau) {
  __shared__ uint32_t hist[1025];
  const int qi = blockIdx.x, tid = threadIdx.x;
  for (int i = tid; i < 1025; i += 256) hist[i] = 0;
  __syncthreads();
  const uint64_t* Lq = lists + (int64_t)qi * nl * K;
  for (int i = tid; i < nl * K; i += 256) {
    const uint64_t key = Lq[i];
    if (key != KEY_NONE) atomicAdd(&hist[(uint32_t)(key >> KEY_ROW_BITS)], 1u);
  }
  __syncthreads();
  if (tid < 64) {  // one wave: prefix sums over 1025 bins, 17 per lane
    int loc = 0;
    for (int j = 0; j < 17; ++j) {
      const int d = tid * 17 + j;
      if (d < 1025) loc += (int)hist[d];
    }
    int inc = loc;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if (tid >= o) inc += y;
    }
    int cum = inc - loc, res = 1025;
    for (int j = 0; j < 17; ++j) {
      const int d = tid * 17 + j;
      if (d < 1025) {
        const int hh = (int)hist[d];
        if (cum < K && cum + hh >= K) res = d;
        cum += hh;
      }
    }
    // exactly one lane (or none) found it
    for (int o = 32; o > 0; o >>= 1) {
      const int y = __shfl_xor(res, o, 64);
      res = y < res ? y : res;
    }
    if (tid == 0) tau[qi] = res;
  }
}

// Suffix candidates -> one sorted list of K keys per query (KEY_NONE padded).
// The matrix-core kernel left, per (query, chunk), a list of keys (v + 1024) << 40 | row and its
// length.  Exact in every case:
//   all lists complete, total <= SUF_CAP  -> sort them all;
//   all lists complete, total  > SUF_CAP  -> histogram of v, threshold T = K-th smallest v, sort
//                                            the keys with v <= T (if they fit);
//   some list overflowed (or neither fits) -> exact rescan of the query's suffix rows.
constexpr int SUF_THREADS = 256;
constexpr int SUF_CAP = 4096;
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
                                                                   int capc, int K, uint64_t* __restrict__ out) {
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
  const int pcq = sh.misc[4];
  const int64_t dfix = (int64_t)pcq - 1024;  // dist = v-field + pc(q) - 1024
  int m = -1;
  bool real_dist = false;
  if (!overflow && total <= SUF_CAP) {
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
  const int np2 = next_pow2(m > 1 ? m : 1);
  for (int i = m + tid; i < np2; i += SUF_THREADS) sh.buf[i] = KEY_NONE;
  __syncthreads();
  block_bitonic_sort_u64(sh.buf, np2);
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

int mfma_plan(int64_t n, int nq, int K, MfmaPlan* p) {
  if (nq < 1 || K < 1 || K > kMfmaMaxK) return VRQ_EUNSUPPORTED;
  int64_t S = n / 16;
  if (S < kMfmaMinPrefix) S = kMfmaMinPrefix;
  if (S > n) S = n;
  p->prefix = S;
  p->nqb = (nq + QPB - 1) / QPB;
  const int64_t rest = n - S;
  int64_t want = 256 / p->nqb;  // one workgroup per CU
  if (want < 1) want = 1;
  int64_t cr = (rest + want - 1) / want;
  cr = (cr + RT - 1) / RT * RT;
  if (cr < RT) cr = RT;
  p->chunk_rows = cr;
  p->nchunks = rest > 0 ? (int)((rest + cr - 1) / cr) : 0;
  // per-(query, chunk) list capacity: 4x the expected hits K * chunk_rows / prefix (iid rows)
  const int64_t expect = (K * cr + S - 1) / S;
  int capc = 64;
  while (capc < 4 * expect && capc < 4096) capc <<= 1;
  p->capc = capc;
  if (scan_plan(S, 128, nq, K, &p->prefix_plan) != VRQ_OK) return VRQ_EUNSUPPORTED;
  if (p->prefix_plan.nchunks + 1 > 4096) return VRQ_EUNSUPPORTED;  // select step's list bound
  p->nl = p->prefix_plan.nchunks + 1;  // prefix chunk lists + the suffix list
  // workspace: prefix lists [nq][nlp][K] | suffix list [nq][K] | cand [nq][nchunks][capc] |
  //            list lengths [nq][nchunks] | tau [nq]
  auto al = [](size_t x) { return (x + 255) & ~size_t(255); };
  p->off_suffix = al(p->prefix_plan.list_bytes);
  p->off_cand = p->off_suffix + al((size_t)nq * K * sizeof(uint64_t));
  p->off_cnt = p->off_cand + al((size_t)nq * p->nchunks * p->capc * sizeof(uint64_t));
  p->off_tau = p->off_cnt + al((size_t)nq * p->nchunks * sizeof(int32_t));
  p->bytes = p->off_tau + (size_t)nq * sizeof(int32_t);
  return VRQ_OK;
}

bool mfma_use(int64_t n, int nq, int K, int flags) {
  if (flags & VRQ_SEARCH_SCAN_VALU) return false;
  const bool ok = K <= kMfmaMaxK && n >= 2 * kMfmaMinPrefix;
  if (flags & VRQ_SEARCH_SCAN_MFMA) return ok;
  return ok && nq >= kMfmaMinQueries;
}

int mfma_scan_launch(const MfmaPlan& p, const uint8_t* codes, int64_t n, const uint8_t* q, int nq, int K,
                     uint8_t* ws, hipStream_t s, int flags) {
  constexpr int ALL = VRQ_SCAN_STAGE_PREFIX | VRQ_SCAN_STAGE_MATRIX | VRQ_SCAN_STAGE_SUFFIX;
  const int st = (flags & ALL) ? (flags & ALL) : ALL;
  uint64_t* lists = (uint64_t*)ws;
  uint64_t* suffix = (uint64_t*)(ws + p.off_suffix);
  uint64_t* cand = (uint64_t*)(ws + p.off_cand);
  int32_t* ccnt = (int32_t*)(ws + p.off_cnt);
  int32_t* tau = (int32_t*)(ws + p.off_tau);
  if (st & VRQ_SCAN_STAGE_PREFIX) {
    int rc = scan_launch(p.prefix_plan, codes, p.prefix, 128, q, nq, K, lists, s);
    if (rc != VRQ_OK) return rc;
    hipLaunchKernelGGL(prefix_tau_kernel, dim3(nq), dim3(256), 0, s, lists, p.prefix_plan.nchunks, K, tau);
    VRQ_LAUNCH_CHECK();
  }
  if ((st & VRQ_SCAN_STAGE_MATRIX) && p.nchunks > 0) {
    hipLaunchKernelGGL(hamming_mfma_kernel, dim3(p.nchunks * p.nqb), dim3(MWAVES * 64), 0, s, codes, n, p.prefix,
                       q, nq, tau, cand, ccnt, p.capc, p.chunk_rows, p.nchunks, p.nqb);
    VRQ_LAUNCH_CHECK();
  }
  if (st & VRQ_SCAN_STAGE_SUFFIX) {
    hipLaunchKernelGGL(suffix_topk_kernel, dim3(nq), dim3(SUF_THREADS), 0, s, codes, n, p.prefix, q, cand, ccnt,
                       p.nchunks, p.capc, K, suffix);
    VRQ_LAUNCH_CHECK();
  }
  return VRQ_OK;
}

}  // namespace vrq
