/*
 * hamming_knn.c -- TEST INFRASTRUCTURE ONLY (checker + timed CPU baseline).
 *
 * Plain-C restatement of FAISS IndexBinaryFlat::search -> hammings_knn_hc
 * (faiss/utils/hamming.cpp; FAISS is an un-vendored, version-unpinned
 * dependency of the reference: dependencies.txt:2 "faiss-cpu"), as reached from
 * CohereEnhancedVectorDB.py:268 (Phase I).  Restated algorithm:
 *   - per query a max-heap of k (dist, id) pairs, initialised to
 *     (INT32_MAX, -1), ordered by (dist, id) (FAISS CMax<int32,int64>::cmp2);
 *   - rows are visited in increasing internal index; a row enters iff
 *     dist < heap_top_dist (strict), replacing the top (heap_replace_top);
 *   - heap_reorder pops the heap into ascending (dist, id) order;
 *   - FAISS parallelises over queries only (OpenMP), so nq = 1 runs on one core.
 * dist = sum over 64-bit words of popcount(q ^ code).
 *
 * Built by oracle/build.sh into oracle/_build/liboracle.so; loaded with ctypes by
 * tests/ and bench.py's cpu_baseline leg only.
 */
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline int gt2(int32_t a, int64_t ia, int32_t b, int64_t ib) {
  return (a > b) || (a == b && ia > ib);
}

/* FAISS heap_replace_top for CMax: root is the largest (dist, id). */
static void heap_replace_top(int k, int32_t* val, int64_t* ids, int32_t v, int64_t id) {
  int32_t* bv = val - 1;
  int64_t* bi = ids - 1;
  int i = 1;
  for (;;) {
    int i1 = i << 1, i2 = i1 + 1;
    if (i1 > k) break;
    if (i2 == k + 1 || gt2(bv[i1], bi[i1], bv[i2], bi[i2])) {
      if (gt2(v, id, bv[i1], bi[i1])) break;
      bv[i] = bv[i1];
      bi[i] = bi[i1];
      i = i1;
    } else {
      if (gt2(v, id, bv[i2], bi[i2])) break;
      bv[i] = bv[i2];
      bi[i] = bi[i2];
      i = i2;
    }
  }
  bv[i] = v;
  bi[i] = id;
}

static void heap_pop(int k, int32_t* val, int64_t* ids) {
  int32_t* bv = val - 1;
  int64_t* bi = ids - 1;
  int32_t v = bv[k];
  int64_t id = bi[k];
  int i = 1;
  for (;;) {
    int i1 = i << 1, i2 = i1 + 1;
    if (i1 > k) break;
    if (i2 == k + 1 || gt2(bv[i1], bi[i1], bv[i2], bi[i2])) {
      if (gt2(v, id, bv[i1], bi[i1])) break;
      bv[i] = bv[i1];
      bi[i] = bi[i1];
      i = i1;
    } else {
      if (gt2(v, id, bv[i2], bi[i2])) break;
      bv[i] = bv[i2];
      bi[i] = bi[i2];
      i = i2;
    }
  }
  bv[i] = v;
  bi[i] = id;
}

/* heap_reorder: ascending (dist, id), valid entries first, missing = (INT32_MAX, -1) */
static void heap_reorder(int k, int32_t* val, int64_t* ids) {
  int i, ii;
  for (i = 0, ii = 0; i < k; i++) {
    int32_t v = val[0];
    int64_t id = ids[0];
    heap_pop(k - i, val, ids);
    val[k - ii - 1] = v;
    ids[k - ii - 1] = id;
    if (id != -1) ii++;
  }
  /* valid entries occupy the last ii slots in ascending order; move them to the front */
  memmove(val, val + k - ii, ii * sizeof(*val));
  memmove(ids, ids + k - ii, ii * sizeof(*ids));
  for (; ii < k; ii++) {
    val[ii] = INT32_MAX;
    ids[ii] = -1;
  }
}

static inline int32_t hamming(const uint64_t* a, const uint64_t* b, int words) {
  int32_t d = 0;
  for (int w = 0; w < words; ++w) d += __builtin_popcountll(a[w] ^ b[w]);
  return d;
}

static inline int32_t hamming128(const uint64_t* a, const uint64_t* b) {
  return __builtin_popcountll(a[0] ^ b[0]) + __builtin_popcountll(a[1] ^ b[1]) +
         __builtin_popcountll(a[2] ^ b[2]) + __builtin_popcountll(a[3] ^ b[3]) +
         __builtin_popcountll(a[4] ^ b[4]) + __builtin_popcountll(a[5] ^ b[5]) +
         __builtin_popcountll(a[6] ^ b[6]) + __builtin_popcountll(a[7] ^ b[7]) +
         __builtin_popcountll(a[8] ^ b[8]) + __builtin_popcountll(a[9] ^ b[9]) +
         __builtin_popcountll(a[10] ^ b[10]) + __builtin_popcountll(a[11] ^ b[11]) +
         __builtin_popcountll(a[12] ^ b[12]) + __builtin_popcountll(a[13] ^ b[13]) +
         __builtin_popcountll(a[14] ^ b[14]) + __builtin_popcountll(a[15] ^ b[15]);
}

/* Returns 0 on success, -1 on bad arguments.  code_bytes must be a multiple of 8. */
int oracle_hamming_knn(const uint8_t* codes, int64_t n, int code_bytes, const uint8_t* queries, int nq, int k,
                       int32_t* D, int64_t* I, int nthreads) {
  if (code_bytes <= 0 || (code_bytes % 8) != 0 || k < 0 || nq < 0 || n < 0) return -1;
  const int words = code_bytes / 8;
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
  for (int q = 0; q < nq; ++q) {
    int32_t* val = D + (int64_t)q * k;
    int64_t* ids = I + (int64_t)q * k;
    for (int i = 0; i < k; ++i) {
      val[i] = INT32_MAX;
      ids[i] = -1;
    }
    if (k == 0) continue;
    const uint64_t* qw = (const uint64_t*)(queries + (int64_t)q * code_bytes);
    if (words == 16) {
      for (int64_t j = 0; j < n; ++j) {
        const int32_t dis = hamming128(qw, (const uint64_t*)(codes + j * 128));
        if (dis < val[0]) heap_replace_top(k, val, ids, dis, j);
      }
    } else {
      for (int64_t j = 0; j < n; ++j) {
        const int32_t dis = hamming(qw, (const uint64_t*)(codes + j * code_bytes), words);
        if (dis < val[0]) heap_replace_top(k, val, ids, dis, j);
      }
    }
    heap_reorder(k, val, ids);
  }
  return 0;
}
