// hamming_scan.hip -- K1: Phase-I exhaustive Hamming scan with per-chunk exact top-K.
//
// Replaces FAISS IndexBinaryFlat::search -> hammings_knn_hc (called from
// CohereEnhancedVectorDB.py:268).  FAISS semantics: a max-heap ordered by
// (dist, id) that admits a row only if dist < heap_top while rows arrive in
// increasing index, i.e. the result is the K smallest rows under the
// lexicographic (dist asc, row asc) order.  Here every wave scans one
// contiguous CHUNK of rows for QG queries and keeps, per query, the exact top-K
// of its chunk under that same order; K2 (select_rescore.hip) merges the chunk
// lists.  The union of chunk top-Ks contains the global top-K, and the merge
// is exact, so the final order is FAISS's.
//
// gfx950 mapping (one wave = one workgroup = one (chunk, query-group)):
//  * corpus rows stream HBM -> LDS with global_load_lds_dwordx4 (LDS-DMA, 1 KiB
//    per wave-instruction, fully coalesced); the per-lane SOURCE address is
//    pre-swizzled so that the row-per-lane ds_read_b128 that follows is
//    bank-conflict-free (linear LDS destination, swizzled source, same XOR on
//    the read).  NBUF tiles in flight per wave.
//  * each lane owns one row (CB/4 dwords in VGPRs); query dwords are
//    wave-uniform and come from scalar loads (SGPR operands of v_xor_b32), so
//    the distance of one (query,row) pair costs CB/4 v_xor + CB/4 v_bcnt
//    (v_bcnt_u32_b32 accumulates) and nothing else.
//  * top-K per query: a 32-bit LDS key (dist << 20 | chunk-local row) list of
//    capacity CAP >= K + 64 and a wave-uniform threshold; a row is appended iff
//    key < tau (ballot + mbcnt compaction).  When the list would overflow it is
//    sorted by a wave-level bitonic network in registers (shuffles for strides
//    < 64, register swaps above) and cut to K; tau = K-th key.
//  * blockIdx -> (chunk, query group) is XCD-aware: blocks that share an XCD
//    (b % 8) get consecutive linear ids, i.e. the same chunk for different
//    query groups, so re-reads of a chunk hit that XCD's L2.
#include "vrq_internal.h"
#include "vrq_scan.h"

namespace vrq {

constexpr int LOCAL_BITS = 20;
constexpr uint32_t LOCAL_MASK = (1u << LOCAL_BITS) - 1;

// Wave-level bitonic sort (ascending) of the CAP u32 keys at buf[0..CAP);
// entries at index >= cnt are treated as +inf.  Result written back to buf.
template <int CAP>
__device__ __forceinline__ void wave_sort_keys(uint32_t* buf, int cnt) {
  constexpr int E = CAP / WAVE;
  int l = lane_id();
  // opaque lane id: keeps the network's lane masks from being hoisted into the scan
  // loop, where they would hold ~100 SGPRs live and push the resident query words out
  asm volatile("" : "+v"(l));
  uint32_t v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int i = e * WAVE + l;
    v[e] = (i < cnt) ? buf[i] : 0xffffffffu;
  }
#pragma unroll
  for (int size = 2; size <= CAP; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= WAVE) {
        const int es = stride / WAVE;
#pragma unroll
        for (int e = 0; e < E; ++e) {
          if ((e & es) == 0) {
            const int i = e * WAVE + l;
            const bool up = (i & size) == 0;
            const uint32_t a = v[e], b = v[e + es];
            const uint32_t mn = a < b ? a : b, mx = a < b ? b : a;
            v[e] = up ? mn : mx;
            v[e + es] = up ? mx : mn;
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const int i = e * WAVE + l;
          const uint32_t p = shfl_xor_u32(v[e], stride);
          const bool up = (i & size) == 0;
          const bool lower = (l & stride) == 0;
          const uint32_t mn = v[e] < p ? v[e] : p, mx = v[e] < p ? p : v[e];
          v[e] = (lower == up) ? mn : mx;
        }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) buf[e * WAVE + l] = v[e];
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef uint32_t v16u __attribute__((ext_vector_type(16)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const void*)p);
}

// 128 query bytes -> 32 SGPRs (two s_load_dwordx16 from the scalar cache) and the
// wait, in ONE asm statement: the SGPRs are valid at ASMEND, so hipcc can neither
// hoist the loads out of the tile loop (that spilled QG*32 SGPRs) nor copy or
// spill the destinations before the data lands.
__device__ __forceinline__ void load_q(v16u& a, v16u& b, const uint8_t* p) {
  asm volatile("s_load_dwordx16 %0, %2, 0x0\n\ts_load_dwordx16 %1, %2, 0x40\n\ts_waitcnt lgkmcnt(0)"
               : "=&s"(a), "=&s"(b)
               : "s"(p)
               : "memory");
}

// d += popcount(q ^ r): v_xor_b32 (SGPR q) + v_bcnt_u32_b32 (bcnt accumulates).  The
// empty asm pins the accumulation order so LLVM does not re-associate the chain
// into bcnt(x,0) + v_add3 trees (+15 % VALU).
__device__ __forceinline__ void xor_bcnt(uint32_t& d, uint32_t q, uint32_t r) {
  d = __popc(q ^ r) + d;
  asm("" : "+v"(d));
}

template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {  // provably wave-uniform (SGPR) pointer
  const uint64_t u = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u), hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_barrier" ::: "memory"); }

// One workgroup = WPG waves scanning one CHUNK of rows for WPG*QG queries; every wave
// owns QG queries (resident in SGPRs for the whole chunk) and the per-query top-K
// state of those queries.  The 64-row tiles stream HBM -> LDS through a 3-deep
// ring shared by the workgroup (each wave issues GLDS/WPG of the 8 LDS-DMA
// instructions of a tile), so a row is fetched once per WPG*QG queries.
template <int QG, int WPG, int CAP>
__global__ __launch_bounds__(64 * WPG) void hamming_scan_kernel(const uint8_t* __restrict__ codes, int64_t n,
                                                                const uint8_t* __restrict__ queries, int nq,
                                                                int K, int64_t chunk_rows, int nchunks, int nqg,
                                                                uint64_t* __restrict__ out) {
  constexpr int CB = 128;             // bytes per 1024-bit code
  constexpr int C = CB / 16;          // 16-byte pieces per row
  constexpr int TILE = 64 * CB;       // bytes per 64-row tile
  constexpr int GLDS = TILE / 1024;   // LDS-DMA wave-instructions per tile (8)
  constexpr int GPW = GLDS / WPG;     // ... issued by each wave
  constexpr int RPG = 16 / C;         // rows per 16-slot bank period
  constexpr int NBUF = 4;
  static_assert(WPG >= 1 && WPG <= GLDS && (GLDS % WPG) == 0, "waves per group");
  static_assert(QG == 1 || QG == 2, "queries per wave");
  static_assert(CAP % WAVE == 0, "cap");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NBUF * TILE + WPG * QG * CAP * 4];

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* cand = reinterpret_cast<uint32_t*>(smem + NBUF * TILE) + wave * QG * CAP;

  // XCD-aware, bijective block -> linear id (blocks b and b+8 share an XCD): blocks of
  // one XCD take consecutive ids = the same chunk for successive query groups (L2 reuse).
  const int nb = gridDim.x, b = blockIdx.x;
  const int xcd = b & 7, slot = b >> 3, q8 = nb >> 3, r8 = nb & 7;
  const int L = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + slot;
  const int chunk = L / nqg;
  const int qg = L - chunk * nqg;
  if (chunk >= nchunks) return;
  const int64_t row0 = (int64_t)chunk * chunk_rows;
  const int64_t row1 = (row0 + chunk_rows < n) ? row0 + chunk_rows : n;
  const int nrows = (int)(row1 - row0);
  const int l = lane_id();
  const int qw0 = (qg * WPG + wave) * QG;                 // first query of this wave
  const int nqa = nq - qw0 < QG ? (nq - qw0 > 0 ? nq - qw0 : 0) : QG;

  // queries -> SGPRs once per chunk (32 SGPRs each)
  v16u qa0, qa1, qb0, qb1;
  const uint8_t* qptr = uniform_ptr(queries + (int64_t)(nqa > 0 ? qw0 : 0) * CB);
  if (nqa > 0) load_q(qa0, qa1, qptr);
  if (QG == 2 && nqa > 1) load_q(qb0, qb1, qptr + CB);

  int cnt[QG];
  uint32_t tau[QG];
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    cnt[j] = 0;
    tau[j] = 0xffffffffu;
  }

  uint32_t raddr[C];  // this lane's row pieces in buffer 0 (swizzled slots)
#pragma unroll
  for (int c = 0; c < C; ++c) raddr[c] = lds_addr(smem) + (uint32_t)((l * C + (c ^ ((l / RPG) % C))) * 16);

  const int ntiles = (nrows + 63) >> 6;
  auto issue = [&](int t) {
    uint8_t* buf = smem + (t % NBUF) * TILE;
    const int64_t tr0 = row0 + (int64_t)t * 64;
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const int gi = wave * GPW + i;
      const int p = gi * 64 + l;
      const int r = p / C, cs = p % C;
      const int c = cs ^ ((r / RPG) % C);
      int64_t row = tr0 + r;
      row = row < row1 ? row : row1 - 1;  // clamp the ragged last tile (lanes masked below)
      __builtin_amdgcn_global_load_lds(codes + row * CB + c * 16,
                                       (__attribute__((address_space(3))) void*)(buf + gi * 1024), 16, 0, 0);
    }
  };
  auto read_tile = [&](int t, v4u (&rv)[C]) {
    const uint32_t boff = (uint32_t)((t % NBUF) * TILE);
#pragma unroll
    for (int c = 0; c < C; ++c)
      asm volatile("ds_read_b128 %0, %1" : "=v"(rv[c]) : "v"(raddr[c] + boff) : "memory");
  };
  auto wait_tile = [&](v4u (&rv)[C]) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(rv[0]), "+v"(rv[1]), "+v"(rv[2]), "+v"(rv[3]), "+v"(rv[4]), "+v"(rv[5]), "+v"(rv[6]),
                   "+v"(rv[7])::"memory");
  };
  // Distances of this lane's row to the wave's (up to) two queries; the two queries'
  // four popcount chains are interleaved for ILP.
  auto distances = [&](const v4u (&rv)[C], uint32_t& da, uint32_t& db) {
    uint32_t a0 = 0, a1 = 0, b0 = 0, b1 = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      xor_bcnt(a0, qa0[4 * c + 0], rv[c].x);
      if (QG == 2) xor_bcnt(b0, qb0[4 * c + 0], rv[c].x);
      xor_bcnt(a1, qa0[4 * c + 1], rv[c].y);
      if (QG == 2) xor_bcnt(b1, qb0[4 * c + 1], rv[c].y);
      xor_bcnt(a0, qa0[4 * c + 2], rv[c].z);
      if (QG == 2) xor_bcnt(b0, qb0[4 * c + 2], rv[c].z);
      xor_bcnt(a1, qa0[4 * c + 3], rv[c].w);
      if (QG == 2) xor_bcnt(b1, qb0[4 * c + 3], rv[c].w);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      xor_bcnt(a0, qa1[4 * c + 0], rv[4 + c].x);
      if (QG == 2) xor_bcnt(b0, qb1[4 * c + 0], rv[4 + c].x);
      xor_bcnt(a1, qa1[4 * c + 1], rv[4 + c].y);
      if (QG == 2) xor_bcnt(b1, qb1[4 * c + 1], rv[4 + c].y);
      xor_bcnt(a0, qa1[4 * c + 2], rv[4 + c].z);
      if (QG == 2) xor_bcnt(b0, qb1[4 * c + 2], rv[4 + c].z);
      xor_bcnt(a1, qa1[4 * c + 3], rv[4 + c].w);
      if (QG == 2) xor_bcnt(b1, qb1[4 * c + 3], rv[4 + c].w);
    }
    da = a0 + a1;
    db = b0 + b1;
  };
  auto accept = [&](int j, uint32_t key) {
    bool acc = key < tau[j];
    uint64_t mask = __ballot(acc);
    if (mask) {
      int nnew = __popcll(mask);
      uint32_t* cj = cand + j * CAP;
      if (cnt[j] + nnew > CAP) {
        wave_sort_keys<CAP>(cj, cnt[j]);
        cnt[j] = cnt[j] < K ? cnt[j] : K;
        if (cnt[j] >= K) tau[j] = __builtin_amdgcn_readfirstlane(cj[K - 1]);
        acc = key < tau[j];
        mask = __ballot(acc);
        nnew = __popcll(mask);
      }
      if (acc) {
        const int pos = cnt[j] + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
        cj[pos] = key;
      }
      cnt[j] += nnew;
    }
  };

  // Software pipeline over a 4-deep LDS ring: while tile t is computed from VGPRs
  // (set A), tile t+1 is read LDS -> VGPRs (set B) and tiles t+2, t+3 are in flight
  // HBM -> LDS.  One workgroup barrier per tile publishes tile t+1 (every wave's DMA
  // pieces waited by that wave's vmcnt) and certifies that every wave finished
  // reading tile t-1, whose buffer (t+3)%4 is then refilled.
  for (int t = 0; t < 3 && t < ntiles; ++t) issue(t);
  if (ntiles > 2)
    wait_vmcnt<2 * GPW>();
  else if (ntiles > 1)
    wait_vmcnt<GPW>();
  else
    wait_vmcnt<0>();
  lds_barrier();
  v4u rA[C], rB[C];
  read_tile(0, rA);
  wait_tile(rA);
  // (The LDS reads of the next tile are issued and retired on every path, the last iteration's
  // included -- where they read a stale ring slot that nothing uses -- so that no read is ever in
  // flight on a path that skips its wait: tests/isa_check.py follows every static path.)
  for (int t = 0; t < ntiles; t += 2) {
    // ---- tile t from A, prefetch t+1 into B
    if (t + 1 < ntiles) {
      if (t + 2 < ntiles) wait_vmcnt<GPW>(); else wait_vmcnt<0>();
      lds_barrier();
    }
    read_tile(t + 1, rB);
    if (t + 3 < ntiles) issue(t + 3);
    {
      const int local = t * 64 + l;
      uint32_t da, db;
      distances(rA, da, db);
      if (nqa > 0) accept(0, local < nrows ? ((da << LOCAL_BITS) | (uint32_t)local) : 0xffffffffu);
      if (QG == 2 && nqa > 1) accept(1, local < nrows ? ((db << LOCAL_BITS) | (uint32_t)local) : 0xffffffffu);
    }
    wait_tile(rB);
    if (t + 1 >= ntiles) break;
    // ---- tile t+1 from B, prefetch t+2 into A
    if (t + 2 < ntiles) {
      if (t + 3 < ntiles) wait_vmcnt<GPW>(); else wait_vmcnt<0>();
      lds_barrier();
    }
    read_tile(t + 2, rA);
    if (t + 4 < ntiles) issue(t + 4);
    {
      const int local = (t + 1) * 64 + l;
      uint32_t da, db;
      distances(rB, da, db);
      if (nqa > 0) accept(0, local < nrows ? ((da << LOCAL_BITS) | (uint32_t)local) : 0xffffffffu);
      if (QG == 2 && nqa > 1) accept(1, local < nrows ? ((db << LOCAL_BITS) | (uint32_t)local) : 0xffffffffu);
    }
    wait_tile(rA);
  }

  // chunk done: exact top-K per query -> global keys (dist << 40 | shard row), padded.
#pragma unroll
  for (int j = 0; j < QG; ++j) {
    if (j >= nqa) break;
    uint32_t* cj = cand + j * CAP;
    wave_sort_keys<CAP>(cj, cnt[j]);
    const int m = cnt[j] < K ? cnt[j] : K;
    uint64_t* o = out + ((int64_t)(qw0 + j) * nchunks + chunk) * K;
    for (int i = l; i < K; i += WAVE) {
      uint64_t gk = KEY_NONE;
      if (i < m) {
        const uint32_t key = cj[i];
        gk = ((uint64_t)(key >> LOCAL_BITS) << KEY_ROW_BITS) | (uint64_t)(row0 + (key & LOCAL_MASK));
      }
      o[i] = gk;
    }
  }
}

// ---------------------------------------------------------------------------
// host side: plan + dispatch
// ---------------------------------------------------------------------------
static int cap_for(int K) {
  int c = 256;
  while (c < K + 64) c <<= 1;
  return c;
}

int scan_plan(int64_t n, int cb, int nq, int K, ScanPlan* p) {
  if (K < 1 || nq < 1 || n < 1) return VRQ_EINVAL;
  if (cb != 128 || K > 1024) return VRQ_EUNSUPPORTED;
  p->cap = cap_for(K);
  p->qg = nq >= 2 ? 2 : 1;
  const int waves_needed = (nq + p->qg - 1) / p->qg;
  int wpg = 1;
  while (wpg < 8 && wpg < waves_needed) wpg <<= 1;
  p->wpg = wpg;
  const int per_group = p->qg * wpg;
  p->nqg = (nq + per_group - 1) / per_group;
  int64_t want = kTargetWaves / ((int64_t)p->nqg * wpg);
  if (want < 1) want = 1;
  int64_t cr = (n + want - 1) / want;
  if (cr < kMinChunkRows) cr = kMinChunkRows;
  cr = (cr + 63) & ~int64_t(63);
  // the merge (select_rescore.hip) takes at most 4096 lists per query
  if ((n + cr - 1) / cr > 4096) cr = ((n + 4095) / 4096 + 63) & ~int64_t(63);
  if (cr > (int64_t(1) << LOCAL_BITS)) cr = int64_t(1) << LOCAL_BITS;  // large batches: more chunks
  if ((n + cr - 1) / cr > 4096) return VRQ_EUNSUPPORTED;                // n > 2^32 rows
  p->chunk_rows = cr;
  p->nchunks = (int)((n + cr - 1) / cr);
  p->list_bytes = (size_t)nq * p->nchunks * K * sizeof(uint64_t);
  return VRQ_OK;
}

template <int QG, int WPG, int CAP>
static int launch_t(const ScanPlan& p, const uint8_t* codes, int64_t n, const uint8_t* q, int nq, int K,
                    uint64_t* lists, hipStream_t s) {
  const int nblocks = p.nchunks * p.nqg;
  hipLaunchKernelGGL((hamming_scan_kernel<QG, WPG, CAP>), dim3(nblocks), dim3(64 * WPG), 0, s, codes, n, q, nq, K,
                     p.chunk_rows, p.nchunks, p.nqg, lists);
  VRQ_LAUNCH_CHECK();
  return VRQ_OK;
}

template <int QG, int CAP>
static int launch_w(const ScanPlan& p, const uint8_t* codes, int64_t n, const uint8_t* q, int nq, int K,
                    uint64_t* lists, hipStream_t s) {
  switch (p.wpg) {
    case 1: return launch_t<QG, 1, CAP>(p, codes, n, q, nq, K, lists, s);
    case 2: return launch_t<QG, 2, CAP>(p, codes, n, q, nq, K, lists, s);
    case 4: return launch_t<QG, 4, CAP>(p, codes, n, q, nq, K, lists, s);
    default: return launch_t<QG, 8, CAP>(p, codes, n, q, nq, K, lists, s);
  }
}

template <int CAP>
static int launch_c(const ScanPlan& p, const uint8_t* codes, int64_t n, const uint8_t* q, int nq, int K,
                    uint64_t* lists, hipStream_t s) {
  return p.qg == 1 ? launch_w<1, CAP>(p, codes, n, q, nq, K, lists, s)
                   : launch_w<2, CAP>(p, codes, n, q, nq, K, lists, s);
}

int scan_launch(const ScanPlan& p, const uint8_t* codes, int64_t n, int cb, const uint8_t* q, int nq, int K,
                uint64_t* lists, hipStream_t s) {
  if (cb != 128) return VRQ_EUNSUPPORTED;
  switch (p.cap) {
    case 256: return launch_c<256>(p, codes, n, q, nq, K, lists, s);
    case 512: return launch_c<512>(p, codes, n, q, nq, K, lists, s);
    case 1024: return launch_c<1024>(p, codes, n, q, nq, K, lists, s);
    case 2048: return launch_c<2048>(p, codes, n, q, nq, K, lists, s);
    default: return VRQ_EUNSUPPORTED;
  }
}

}  // namespace vrq
