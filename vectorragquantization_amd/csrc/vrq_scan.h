// vrq_scan.h -- host-side plan of the Phase-I scan (K1) shared by the C ABI entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/vrq.h"

namespace vrq {

// Waves the scan aims to launch (256 CUs x 16): enough to fill every SIMD several
// times over.  A constant (not a device query) so workspace sizes are pure
// functions of the call shape.
constexpr int64_t kTargetWaves = 4096;
// A chunk emits K candidate keys; >= 4096 rows keeps that output < 0.2 % of the
// bytes the chunk scans (K = 100, 128-byte codes).
constexpr int64_t kMinChunkRows = 4096;

struct ScanPlan {
  int cap;             // per-query LDS candidate capacity (pow2 >= K + 64)
  int qg;              // queries per wave (resident in SGPRs)
  int wpg;             // waves per workgroup (share one LDS tile ring)
  int nqg;             // query groups
  int64_t chunk_rows;  // rows per wave (multiple of 64, <= 2^20)
  int nchunks;
  size_t list_bytes;   // nq * nchunks * K * 8
};

int scan_plan(int64_t n, int cb, int nq, int K, ScanPlan* p);
int scan_launch(const ScanPlan& p, const uint8_t* codes, int64_t n, int cb, const uint8_t* q, int nq, int K,
                uint64_t* lists, hipStream_t s);

// ---- K1m: matrix-core scan for large query batches (hamming_mfma.hip) ----
constexpr int kMfmaMaxK = 128;           // K bound of the path
// the minimum dense sample (VRQ_MIN_SAMPLE: A/B builds).  Round 6: 65 536 rows; with the round-6 suffix and
// finish a looser tau_s costs less than the sample rows it saves (config 2: step 0.459-0.468 -> 0.445-0.450 ms,
// sample pass 0.075 -> 0.048 ms, matrix pass +0.007 ms; profiles/r6_c2_min_sample_ab.jsonl)
#ifndef VRQ_MIN_SAMPLE
#define VRQ_MIN_SAMPLE 65536
#endif
constexpr int64_t kMfmaMinSample = VRQ_MIN_SAMPLE;
constexpr int64_t kMfmaMaxSample = 1 << 20;   // dense-sample cap (1M rows: ~0.3 ms of MFMA at nq = 1024)
constexpr int64_t kMfmaMinRows = 65536;  // below this the wavefront scan is used
constexpr int kMfmaMinQueries = 1;       // auto-selection threshold on the batch size (K1r below 129)
// dense threshold sample = n / kMfmaSampleDiv rows (clamped above).  Per-step time at nq = 1024
// (profiles/r3_c4_shard_sample_div.txt): 12.5M rows (one rank of 8) div 16 / 32 / 64 / 128 = 4.31 /
// 4.22 / 4.23 / 4.32 ms, 25M rows 8.00 / 7.96 / 7.90 / 8.11 ms; 100M and 1M rows are at the clamps
constexpr int64_t kMfmaSampleDiv = 32;

struct MfmaPlan {
  int64_t sample;            // dense sample rows (sample_chunks * sample_chunk_rows)
  int64_t dvcols;            // dv columns per query: 32 lane minima per sample chunk
  int64_t sample_chunk_rows;
  int64_t sample_stride;     // sample chunk c starts at row c * sample_stride
  int64_t sample_tile_stride;  // rows between consecutive sample tiles (>= 64)
  int sample_chunks;
  int j;                     // sampled threshold order (tau_s = d_(j) + 1); K = tau_p only
  int capc;                  // candidate capacity per (query, chunk) list
  int rows;                  // 1: the row-split small-batch kernel K1r (nq <= 128, nqb = 1)
  int swap;                  // the large-batch pass runs K1s (row sets resident) instead of K1m (MB = 4):
                             // 1 = K1s<2, 8> (two waves per SIMD), 2 = K1s<4, 4> (one wave per SIMD)
  int rows_sample;           // 1: K1r also runs the dense sample pass (MB <= 2, nq <= 64)
  int mb;                    // M-blocks (32 queries) per wave of the matrix kernel: 4 or 2 (K1r: 1, 2 (lean), 4)
  int qpb;                   // queries per workgroup (128 * mb)
  int nqb;                   // query blocks of the thresholded pass
  int nqb_s;                 // query blocks of the dense sample pass (always the MB = 2 kernel)
  int64_t chunk_rows;        // rows per workgroup of the thresholded pass (multiple of 64)
  int nchunks;
  size_t off_suffix, off_cand, off_cnt, off_tau, bytes;
};

int mfma_plan(int64_t n, int nq, int K, MfmaPlan* p);
bool mfma_use(int64_t n, int nq, int K, int flags);
int mfma_scan_launch(const MfmaPlan& p, const uint8_t* codes, int64_t n, const uint8_t* q, int nq, int K,
                     uint8_t* ws, hipStream_t s, int flags);

}  // namespace vrq
