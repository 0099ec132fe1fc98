// Times hamming_mfma_kernel alone on a random 10M-row corpus, nq = 1024, with parts removed
// at compile time (VRQ_BISECT: 1 epilogue, 2 unpack, 4 MFMA) to locate its bottleneck.
// Build: tools/probes/build_bisect.sh.  Prints one JSON line.
#include "../../vectorragquantization_amd/csrc/hamming_mfma.hip"
#include <stdio.h>

__global__ void fill(uint32_t* p, int64_t n, uint32_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = x;
  }
}
__global__ void setv(int32_t* p, int n, int v) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
  const int nq = argc > 2 ? atoi(argv[2]) : 1024;
  const int tauv = argc > 3 ? atoi(argv[3]) : 440;
  vrq::MfmaPlan p;
  if (vrq::mfma_plan(n, nq, 100, &p) != VRQ_OK) return 2;
  uint8_t *codes, *q, *ws;
  int32_t* tau;
  (void)hipMalloc(&codes, n * 128);
  (void)hipMalloc(&q, (size_t)nq * 128);
  (void)hipMalloc(&ws, p.bytes);
  (void)hipMalloc(&tau, nq * 4);
  hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)codes, n * 32, 1u);
  hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, 0, (uint32_t*)q, (int64_t)nq * 32, 7u);
  hipLaunchKernelGGL(setv, dim3((nq + 255) / 256), dim3(256), 0, 0, tau, nq, tauv);
  uint64_t* cand = (uint64_t*)(ws + p.off_cand);
  int32_t* ccnt = (int32_t*)(ws + p.off_cnt);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int it = 0; it < 6; ++it) {
    (void)hipEventRecord(e0, 0);
    if (p.mb == 4)
      hipLaunchKernelGGL((vrq::hamming_mfma_kernel<vrq::MFMA_MAIN, 4>), dim3(p.nchunks * p.nqb), dim3(vrq::MWAVES * 64), 0,
                         0, codes, n, (int64_t)0, q, nq, tau, cand, ccnt, p.capc, p.chunk_rows, p.chunk_rows, (int64_t)vrq::RT, p.nchunks,
                         p.nqb, (const int32_t*)nullptr, (const int32_t*)nullptr, (uint16_t*)nullptr, (int64_t)0);
    else
      hipLaunchKernelGGL((vrq::hamming_mfma_kernel<vrq::MFMA_MAIN, 2>), dim3(p.nchunks * p.nqb), dim3(vrq::MWAVES * 64), 0,
                         0, codes, n, (int64_t)0, q, nq, tau, cand, ccnt, p.capc, p.chunk_rows, p.chunk_rows, (int64_t)vrq::RT, p.nchunks,
                         p.nqb, (const int32_t*)nullptr, (const int32_t*)nullptr, (uint16_t*)nullptr, (int64_t)0);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (it > 0 && ms < best) best = ms;
  }
  const double rows = (double)n;
  const double tiles_per_wg = (double)p.chunk_rows / vrq::RT;
  const double ops = rows * nq * 2048.0;
  printf("{\"mb\": %d, \"bisect\": %d, \"n\": %lld, \"nq\": %d, \"ms\": %.4f, \"us_per_tile\": %.3f, \"TOPS\": %.1f, "
         "\"mfma_frac_fp4_dense_10066\": %.3f}\n",
         p.mb, VRQ_BISECT, (long long)n, nq, best, best * 1e3 / tiles_per_wg, ops / (best * 1e-3) / 1e12,
         ops / (best * 1e-3) / 1e12 / 10066.0);
  return 0;
}
