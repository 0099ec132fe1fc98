// vrq_scan.h -- host-side plan of the Phase-I scan (K1) shared by the C ABI entry points.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

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

}  // namespace vrq
