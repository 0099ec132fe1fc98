"""NumPy restatement of the reference hot path -- TEST INFRASTRUCTURE ONLY.

See ``oracle/__init__.py`` for the usage rule (checker / CPU baseline only).
Every function cites the reference ``file:line`` it restates; paths are
relative to the reference checkout (aitrailblazer/VectorRAGQuantization @
2025-02-18).  FAISS is not vendored in the reference; its semantics are
restated from ``IndexBinaryFlat::search`` -> ``hammings_knn_hc`` (heap top-k,
insert iff ``dis < heap_top``, heap ordered by (dist, id), final reorder).
"""
from __future__ import annotations

import numpy as np

INT32_MAX = np.iinfo(np.int32).max

# byte -> popcount table (Phase I restatement)
_POPCNT8 = np.array([bin(i).count("1") for i in range(256)], dtype=np.int32)


# --------------------------------------------------------------------------
# Phase I: FAISS IndexBinaryFlat / IndexBinaryIDMap2 restatement
# --------------------------------------------------------------------------
def hamming_distances(codes: np.ndarray, queries: np.ndarray, chunk: int = 8192) -> np.ndarray:
    """All-pairs Hamming distance, i32[nq, n].

    Restates ``hc.hamming(bs2_)`` of FAISS ``hammings_knn_hc`` reached from
    ``CohereEnhancedVectorDB.py:268``: popcount(q XOR code) over the packed
    ``ubinary`` bytes (bit order is irrelevant for Hamming).
    """
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    queries = np.ascontiguousarray(queries, dtype=np.uint8)
    nq, n = queries.shape[0], codes.shape[0]
    out = np.empty((nq, n), dtype=np.int32)
    for s in range(0, n, chunk):
        c = codes[s:s + chunk]
        x = queries[:, None, :] ^ c[None, :, :]
        out[:, s:s + chunk] = _POPCNT8[x].sum(axis=2, dtype=np.int32)
    return out


def binary_flat_search(codes: np.ndarray, queries: np.ndarray, k: int):
    """FAISS ``IndexBinaryFlat::search`` restatement -> (D i32[nq,k], I i64[nq,k]).

    ``hammings_knn_hc`` keeps a max-heap ordered by (dist, id), inserts a row
    only if ``dis < heap_top`` (strict) while rows arrive in increasing
    internal index, and ``heap_reorder`` emits ascending (dist, id).  The result
    is therefore the k smallest rows under the lexicographic (dist asc,
    internal index asc) order; missing slots (n < k) are (INT32_MAX, -1).
    Call site: ``CohereEnhancedVectorDB.py:267-268``.
    """
    nq = queries.shape[0]
    n = codes.shape[0]
    D = np.full((nq, k), INT32_MAX, dtype=np.int32)
    I = np.full((nq, k), -1, dtype=np.int64)
    if n == 0 or k == 0:
        return D, I
    dist = hamming_distances(codes, queries)
    kk = min(k, n)
    idx = np.arange(n, dtype=np.int64)
    for q in range(nq):
        order = np.lexsort((idx, dist[q]))[:kk]
        D[q, :kk] = dist[q][order]
        I[q, :kk] = order
    return D, I


class IndexBinaryIDMap2:
    """NumPy restatement of ``faiss.IndexBinaryIDMap2(faiss.IndexBinaryFlat(d))``.

    Only the protocol the reference exercises: ``add_with_ids``
    (``CohereEnhancedVectorDB.py:217``), ``search`` (``:268``),
    ``reconstruct`` (``:286``), ``remove_ids`` (``:334``), ``ntotal``
    (``:247,267,350``).  ``remove_ids`` compacts storage preserving the order
    of survivors; ``rev_map`` maps an external id to its (last added) row.
    """

    def __init__(self, d: int = 1024):
        self.d = d
        self.code_size = d // 8
        self.xb = np.zeros((0, self.code_size), dtype=np.uint8)
        self.id_map = np.zeros((0,), dtype=np.int64)
        self.rev_map: dict[int, int] = {}

    @property
    def ntotal(self) -> int:
        return int(self.xb.shape[0])

    def add_with_ids(self, x: np.ndarray, ids: np.ndarray) -> None:
        x = np.ascontiguousarray(x, dtype=np.uint8).reshape(-1, self.code_size)
        ids = np.asarray(ids, dtype=np.int64).reshape(-1)
        base = self.ntotal
        self.xb = np.concatenate([self.xb, x], axis=0)
        self.id_map = np.concatenate([self.id_map, ids])
        for j, e in enumerate(ids.tolist()):
            self.rev_map[e] = base + j

    def search(self, q: np.ndarray, k: int):
        D, I = binary_flat_search(self.xb, np.asarray(q, dtype=np.uint8).reshape(-1, self.code_size), k)
        L = np.where(I >= 0, self.id_map[np.maximum(I, 0)] if self.ntotal else -1, -1)
        return D, L.astype(np.int64)

    def reconstruct(self, key) -> np.ndarray:
        return self.xb[self.rev_map[int(key)]].copy()

    def remove_ids(self, ids) -> int:
        rm = set(int(i) for i in np.asarray(ids).reshape(-1).tolist())
        keep = np.array([int(e) not in rm for e in self.id_map.tolist()], dtype=bool)
        nrm = int((~keep).sum())
        self.xb = self.xb[keep]
        self.id_map = self.id_map[keep]
        self.rev_map = {int(e): j for j, e in enumerate(self.id_map.tolist())}
        return nrm


# --------------------------------------------------------------------------
# Phases II / III: literal restatement of CohereEnhancedVectorDB.search
# --------------------------------------------------------------------------
def three_phase_search(index: IndexBinaryIDMap2, doc_int8: dict, doc_text: dict,
                       query_float: np.ndarray, query_ubinary: np.ndarray,
                       k: int = 10, binary_oversample: int = 10,
                       int8_oversample: int = 3) -> list:
    """Per-query restatement of ``CohereEnhancedVectorDB.search`` (``:227-322``).

    ``doc_int8`` maps external id -> int8[d] (the RocksDict ``"int8"`` value,
    ``:221,303-307``), ``doc_text`` maps id -> text.  Arithmetic follows the
    reference exactly: Phase II ``float32 . int32 -> float64`` dot over
    ``2*unpackbits-1`` (``:286-290``), Phase III ``float(float32 . int8)`` /
    ``np.linalg.norm(int8)`` (float64) with ``-inf`` for a zero norm
    (``:307-313``), Python's stable sorts (``:274,296,321``).
    """
    if index.ntotal == 0:                                          # :247-249
        return []
    qf = np.asarray(query_float, dtype=np.float32).reshape(1, -1)  # :260
    qb = np.asarray(query_ubinary, dtype=np.uint8).reshape(1, -1)  # :261
    binary_k = min(k * binary_oversample, index.ntotal)            # :267
    distances, ids = index.search(qb, binary_k)                    # :268
    hits = [{"doc_id": int(i), "score_hamming": int(d)}
            for i, d in zip(ids[0], distances[0]) if i != -1]      # :269-273
    hits.sort(key=lambda h: h["score_hamming"])                    # :274
    cands = hits[:k * binary_oversample]                           # :275
    if not cands:
        return []
    for h in cands:                                                # :283-293
        bits = np.unpackbits(index.reconstruct(h["doc_id"]), axis=-1).astype(np.int32)
        h["score_binary"] = float(qf[0].dot(2 * bits - 1))
    cands.sort(key=lambda h: h["score_binary"], reverse=True)      # :296
    resc = cands[:k * int8_oversample]                             # :297
    final = []
    for h in resc:                                                 # :302-318
        v = doc_int8.get(h["doc_id"])
        if v is None:
            continue
        v = np.asarray(v, dtype=np.int8)
        nrm = np.linalg.norm(v)
        h["score_cosine"] = -np.inf if nrm == 0 else float(qf[0].dot(v)) / nrm
        h["doc"] = doc_text.get(h["doc_id"], "N/A")
        final.append(h)
    final.sort(key=lambda h: h["score_cosine"], reverse=True)      # :321
    return final[:k]                                               # :322


def three_phase_batch(codes: np.ndarray, int8: np.ndarray, ids: np.ndarray,
                      qf: np.ndarray, qb: np.ndarray, k: int = 10,
                      binary_oversample: int = 10, int8_oversample: int = 3, phase1=None):
    """Array form of ``three_phase_search`` for many queries (oracle for the GPU path).

    ``phase1`` = (D, I) of the Phase-I top-``k * binary_oversample`` when already computed (e.g. by
    the C restatement of hammings_knn_hc for a large corpus); otherwise ``binary_flat_search``.

    Rows are internal indices (insertion order); ``ids`` is the id map.
    Returns per query a dict of arrays: ``row`` (internal index), ``doc_id``,
    ``hamming``, ``binary``, ``cosine`` for the final top-k, plus the
    intermediate ``p1_rows``/``p1_dist`` (Phase I), ``p2_rows``/``p2_score``
    (Phase II, in stable-sorted order).  Phase II uses a float64 GEMV (exact:
    every partial sum of float32 values of an embedding fits in 53 bits, so
    the result equals the reference's per-candidate ``ddot``); Phase III uses
    float32 ``sdot`` per candidate exactly like ``:312``.
    """
    n = codes.shape[0]
    out = []
    if n == 0:
        return [None] * qf.shape[0]
    binary_k = min(k * binary_oversample, n)
    D, I = binary_flat_search(codes, qb, binary_k) if phase1 is None else phase1
    norms = int8_row_norms(int8)
    for q in range(qf.shape[0]):
        rows = I[q][I[q] >= 0]
        dist = D[q][: rows.shape[0]]
        pm = 2 * np.unpackbits(codes[rows], axis=1).astype(np.int32) - 1
        s2 = pm.astype(np.float64) @ qf[q].astype(np.float64)
        o2 = sorted(range(rows.shape[0]), key=lambda j: -s2[j])   # stable, desc
        o2 = np.array(o2[: k * int8_oversample], dtype=np.int64)
        r3 = rows[o2]
        s3 = np.empty(r3.shape[0], dtype=np.float64)
        for j, r in enumerate(r3.tolist()):
            nrm = norms[r]
            s3[j] = -np.inf if nrm == 0 else float(qf[q].dot(int8[r])) / nrm
        o3 = np.array(sorted(range(r3.shape[0]), key=lambda j: -s3[j])[:k], dtype=np.int64)
        fin = o2[o3]
        out.append({
            "p1_rows": rows, "p1_dist": dist,
            "p2_score_by_p1": s2,
            "p2_order": o2,
            "row": rows[fin], "doc_id": ids[rows[fin]], "hamming": dist[fin],
            "binary": s2[fin], "cosine": s3[o3],
        })
    return out


def exhaustive_scores(mode: str, qf: np.ndarray, codes: np.ndarray = None, x8: np.ndarray = None) -> np.ndarray:
    """Reference Phase-II or Phase-III score of EVERY row for each query (config 5), f64 [nq, n].

    ``"binary"``: ``float(q . (2*unpackbits(code)-1))`` with the float32 query promoted to float64
    (``CohereEnhancedVectorDB.py:283-293``; every product is +-q_i, so the float64 GEMV equals the
    reference's per-candidate ddot).  ``"int8_cosine"``: ``float32(q . int8) / ||int8||``, -inf for
    a zero norm (``:302-318``), with the float32 dot taken as the correctly rounded exact dot (the
    GPU's definition; NumPy's sdot is within a few ulps of it).
    """
    q64 = np.asarray(qf, dtype=np.float32).astype(np.float64)
    n = (codes if mode == "binary" else x8).shape[0]
    out = np.empty((q64.shape[0], n), dtype=np.float64)
    for a in range(0, n, 16384):                      # row blocks: bounded host memory
        b = min(n, a + 16384)
        if mode == "binary":
            pm = (2 * np.unpackbits(codes[a:b], axis=1).astype(np.int8) - 1).astype(np.float64)
            out[:, a:b] = q64 @ pm.T
            continue
        xb = np.asarray(x8[a:b])
        dot = (q64 @ xb.astype(np.float64).T).astype(np.float32).astype(np.float64)
        nrm = int8_row_norms(xb)
        with np.errstate(divide="ignore", invalid="ignore"):
            sb = dot / nrm[None, :]
        sb[:, nrm == 0] = -np.inf
        out[:, a:b] = sb
    return out


def exhaustive_topk(scores: np.ndarray, k: int):
    """Top-k rows per query of an [nq, n] score matrix in the reference's order: Python's stable
    ``sorted(..., reverse=True)`` over the rows in index order, i.e. (score desc, row asc)."""
    n = scores.shape[1]
    rows = np.arange(n)
    out = []
    for q in range(scores.shape[0]):
        o = np.lexsort((rows, -scores[q]))[: min(k, n)]
        out.append(o)
    return np.array(out, dtype=np.int64)


def dequantize(mode: str, q: np.ndarray, minmax: np.ndarray = None, limit: float = None, dim: int = 1024):
    """Restatement of the VectorDB* ``_dequantize_*`` methods for a batch of rows (f32[n, dim]):
    ``int8g`` VectorDBInt8Global.py:144-152, ``int16g`` VectorDBInt16Global.py:144-152, ``int4g``
    VectorDBInt4Global.py:166-188, ``int8`` VectorDBInt8.py:129-138, ``int4`` VectorDBInt4.py:157-184."""
    q = np.asarray(q)
    if mode == "int8g":
        return q.astype(np.float32) * np.float32(limit / 127.0)
    if mode == "int16g":
        return q.astype(np.float32) * np.float32(limit / 32767.0)
    if mode in ("int4g", "int4"):
        b = q.view(np.uint8).astype(np.int64)
        nib = np.stack([(b >> 4) & 15, b & 15], axis=-1).reshape(q.shape[0], -1)[:, :dim]
        if mode == "int4g":
            return ((nib - 8) * (limit / 7.0)).astype(np.float32)
        out = np.zeros((q.shape[0], dim), np.float32)
        for r in range(q.shape[0]):
            mn, mx = float(minmax[r, 0]), float(minmax[r, 1])
            if mn != mx:
                out[r] = ((nib[r] - 8) * (max(abs(mn), abs(mx)) / 7.0)).astype(np.float32)
        return out
    out = np.zeros(q.shape, np.float32)                      # "int8": np.float32 min / max
    for r in range(q.shape[0]):
        mn, mx = np.float32(minmax[r, 0]), np.float32(minmax[r, 1])
        if mn != mx:
            scale = np.float32(max(abs(mn), abs(mx)) / np.float32(127))
            out[r] = q[r].astype(np.float32) * scale
    return out


def dequant_scores(qf: np.ndarray, deq: np.ndarray) -> np.ndarray:
    """``float(np.dot(query_float, doc_emb))`` (VectorDBInt8Global.py:235) for every (query, row),
    f64 [nq, n]: the float32 dot taken as the correctly rounded exact dot (the GPU's definition;
    NumPy's sdot is within a few ulps of it)."""
    return (np.asarray(qf, np.float32).astype(np.float64) @ np.asarray(deq, np.float32).astype(np.float64).T
            ).astype(np.float32).astype(np.float64)


def int8_row_norms(x: np.ndarray) -> np.ndarray:
    """``np.linalg.norm(doc_int8)`` per row (float64), ``CohereEnhancedVectorDB.py:308``."""
    x = np.asarray(x)
    return np.sqrt((x.astype(np.float64) ** 2).sum(axis=1)) if x.ndim == 2 else np.linalg.norm(x)


def float_ip_topk(F: np.ndarray, Q: np.ndarray, k: int) -> np.ndarray:
    """Exact float32 inner-product top-k ids (``CohereVectorDBFloat`` ground truth,
    ``CohereVectorDBFloat.py:62,156``).  Ties by lower row (FAISS CMin heap)."""
    S = Q.astype(np.float32) @ F.astype(np.float32).T
    out = np.empty((Q.shape[0], k), dtype=np.int64)
    idx = np.arange(F.shape[0])
    for q in range(Q.shape[0]):
        out[q] = np.lexsort((idx, -S[q]))[:k]
    return out


def flat_ip_scores(F: np.ndarray, Q: np.ndarray) -> np.ndarray:
    """IndexFlatIP scores q . x (``CohereVectorDBFloat.py:62,156``) for every (query, row), f64
    [nq, n] holding float32 values: the exact f64 dot rounded once to float32 (the GPU's
    definition; FAISS's sgemm rounds per step and lands within the float32 summation error)."""
    return (np.asarray(Q, np.float32).astype(np.float64) @ np.asarray(F, np.float32).astype(np.float64).T
            ).astype(np.float32).astype(np.float64)


def flat_ip_search(F: np.ndarray, Q: np.ndarray, k: int, chunk: int = 64):
    """FAISS ``IndexFlatIP.search`` restated: per query the k largest ``flat_ip_scores`` ordered
    (score desc, row asc) -- FAISS's result order for IP; the reference then re-sorts stably by
    score (``CohereVectorDBFloat.py:170``), which keeps it.  Returns (scores f64[nq, k'], rows
    i64[nq, k']) with k' = min(k, n)."""
    F = np.asarray(F, np.float32)
    Q = np.asarray(Q, np.float32).reshape(-1, F.shape[1])
    kk = min(k, F.shape[0])
    rows = np.empty((Q.shape[0], kk), np.int64)
    sc = np.empty((Q.shape[0], kk), np.float64)
    idx = np.arange(F.shape[0])
    for c in range(0, Q.shape[0], chunk):
        S = flat_ip_scores(F, Q[c:c + chunk])
        for j in range(S.shape[0]):
            o = np.lexsort((idx, -S[j]))[:kk]
            rows[c + j] = o
            sc[c + j] = S[j, o]
    return sc, rows


class IndexFlatIPIDMap:
    """NumPy restatement of ``faiss.IndexIDMap(faiss.IndexFlatIP(d))`` as the reference drives it
    (``CohereVectorDBFloat.py:62`` build, ``:133`` add_with_ids, ``:156`` search, ``:177``
    remove_ids): rows in insertion order, ``remove_ids`` compacts keeping the survivors' order,
    labels are ``id_map[row]``, -1 past ntotal."""

    def __init__(self, d: int = 1024):
        self.d = d
        self.xb = np.zeros((0, d), np.float32)
        self.id_map = np.zeros((0,), np.int64)

    @property
    def ntotal(self) -> int:
        return int(self.xb.shape[0])

    def add_with_ids(self, x, ids) -> None:
        self.xb = np.concatenate([self.xb, np.asarray(x, np.float32).reshape(-1, self.d)])
        self.id_map = np.concatenate([self.id_map, np.asarray(ids, np.int64).reshape(-1)])

    def search(self, q, k: int):
        q = np.asarray(q, np.float32).reshape(-1, self.d)
        D = np.full((q.shape[0], k), -np.finfo(np.float32).max, np.float32)
        L = np.full((q.shape[0], k), -1, np.int64)
        if self.ntotal:
            sc, rows = flat_ip_search(self.xb, q, k)
            D[:, :rows.shape[1]] = sc.astype(np.float32)
            L[:, :rows.shape[1]] = self.id_map[rows]
        return D, L

    def remove_ids(self, ids) -> int:
        keep = ~np.isin(self.id_map, np.asarray(ids, np.int64))
        self.xb, self.id_map = self.xb[keep], self.id_map[keep]
        return int((~keep).sum())


# --------------------------------------------------------------------------
# Encoders (VectorDBInt{4,8,16}{,Global}); literal restatements
# --------------------------------------------------------------------------
def to_binary(x: np.ndarray) -> np.ndarray:
    """``_to_binary``: packbits(x > np.mean(x)) -- ``VectorDBInt8Global.py:154-160``
    (identical in ``VectorDBInt8.py:140-146``, ``VectorDBInt4.py:186-192``,
    ``VectorDBInt4Global.py:190-196``, ``VectorDBInt16Global.py:154-160``,
    ``VectorDBInt16.py:148-157`` where the mean of int16 is float64)."""
    return np.packbits((x > np.mean(x)).astype(np.uint8))


def to_binary_sign(x: np.ndarray) -> np.ndarray:
    """Cohere ``ubinary`` emulation for synthetic corpora: packbits(x > 0).
    (Matches the real ``db_cohere_enhanced`` codes vs ``db_cohere_float`` floats
    on all but 2 of 1,024,000 bits)"""
    return np.packbits((x > 0).astype(np.uint8))


def quantize_int8_global(x: np.ndarray, limit: float) -> np.ndarray:
    """``VectorDBInt8Global._quantize_to_int8`` (``VectorDBInt8Global.py:130-142``)."""
    clipped = np.clip(x, -limit, limit)
    scale = 127.0 / limit
    scaled = np.round(clipped * scale)
    return np.clip(scaled, -127, 127).astype(np.int8)


def quantize_int16_global(x: np.ndarray, limit: float) -> np.ndarray:
    """``VectorDBInt16Global._quantize_to_int16`` (``VectorDBInt16Global.py:130-142``)."""
    clipped = np.clip(x, -limit, limit)
    scale = 32767.0 / limit
    scaled = np.round(clipped * scale)
    return np.clip(scaled, -32767, 32767).astype(np.int16)


def _pack_int4(scaled: np.ndarray) -> np.ndarray:
    # nibble loop of VectorDBInt4.py:138-153 / VectorDBInt4Global.py:150-164
    n = scaled.shape[0]
    lp = (n + 1) // 2
    out = np.zeros(lp, dtype=np.int8)
    for i in range(lp):
        a = int(scaled[2 * i]) + 8
        b = int(scaled[2 * i + 1]) + 8 if 2 * i + 1 < n else 0
        c = ((a & 0x0F) << 4) | (b & 0x0F)
        if c > 127:
            c -= 256
        out[i] = np.int8(c)
    return out


def quantize_int4_global(x: np.ndarray, limit: float) -> np.ndarray:
    """``VectorDBInt4Global._quantize_to_int4`` (``VectorDBInt4Global.py:129-164``).
    Reproduces the reference bug: ``limit`` is ignored, the scale is the
    per-vector 7/max|x|."""
    mn = float(np.min(x))
    mx = float(np.max(x))
    if mx == mn:
        return np.zeros((x.shape[0] + 1) // 2, dtype=np.int8)
    scale = 7.0 / max(abs(mn), abs(mx))
    scaled = np.clip(np.round(x * scale), -8, 7).astype(np.int8)
    return _pack_int4(scaled)


def quantize_int8_local(x: np.ndarray):
    """``VectorDBInt8._quantize_to_int8`` (``VectorDBInt8.py:114-126``):
    scale = 127/max(|min|,|max|) in float32, truncating ``astype(int8)``."""
    mn = np.min(x)
    mx = np.max(x)
    if mx == mn:
        return np.zeros_like(x, dtype=np.int8), mn, mx
    scale = 127 / max(abs(mn), abs(mx))
    return (x * scale).astype(np.int8), mn, mx


def quantize_int4_local(x: np.ndarray):
    """``VectorDBInt4._quantize_to_int4`` (``VectorDBInt4.py:116-154``)."""
    mn = float(np.min(x))
    mx = float(np.max(x))
    if mx == mn:
        return np.zeros((x.shape[0] + 1) // 2, dtype=np.int8), mn, mx
    scale = 7.0 / max(abs(mn), abs(mx))
    scaled = np.clip(np.round(x * scale), -8, 7).astype(np.int8)
    return _pack_int4(scaled), mn, mx


def dequantize_int8_global(q: np.ndarray, limit: float) -> np.ndarray:
    """``VectorDBInt8Global._dequantize_int8`` (``:144-152``)."""
    return q.astype(np.float32) * (limit / 127.0)


def encode_batch(mode: str, X: np.ndarray, limit: float = 0.3):
    """Row-wise application of one encoder; returns (codes, quantized, minmax|None)."""
    X = np.asarray(X)
    codes, qs, mm = [], [], []
    for x in X:
        if mode == "int8g":
            qs.append(quantize_int8_global(x, limit)); codes.append(to_binary(x))
        elif mode == "int16g":
            qs.append(quantize_int16_global(x, limit)); codes.append(to_binary(x))
        elif mode == "int4g":
            qs.append(quantize_int4_global(x, limit)); codes.append(to_binary(x))
        elif mode == "int8":
            q, a, b = quantize_int8_local(x); qs.append(q); mm.append((a, b)); codes.append(to_binary(x))
        elif mode == "int4":
            q, a, b = quantize_int4_local(x); qs.append(q); mm.append((a, b)); codes.append(to_binary(x))
        elif mode == "bin16":
            codes.append(to_binary(x))
        elif mode == "cohere":
            qs.append(quantize_int8_global(x, limit)); codes.append(to_binary_sign(x))
        else:
            raise ValueError(mode)
    codes = np.stack(codes) if codes else np.zeros((0, X.shape[1] // 8), np.uint8)
    qs = np.stack(qs) if qs else None
    mm = np.array(mm, dtype=np.float64) if mm else None
    return codes, qs, mm


# --------------------------------------------------------------------------
# VectorDBInt{4,8,16}{,Global}: add_documents / remove_document / search
# --------------------------------------------------------------------------
class QuantVectorDB:
    """Restatement of the six VectorDB* classes' document store + search (float vectors in, no HTTP):
    ``add`` = ``add_documents`` without the embedding call (dedupe by remove, ``add_with_ids`` of the
    ``_to_binary`` codes, doc store ``{id: (quantised row, min_max, float row)}`` keyed by id, the last
    write wins -- e.g. ``VectorDBInt8Global.py:162-203``); ``search`` = ``:205-252`` (Phase I
    top-``min(k * os, ntotal)``, ``float(np.dot(query_float, doc_emb))`` with ``doc_emb`` the
    dequantised row or the float row (``compare_float32``), stable sort by score desc, first k);
    ``bin16`` = ``VectorDBInt16.py:221-263`` (Hamming order, score = distance)."""

    def __init__(self, mode: str, limit: float = 0.0, dim: int = 1024):
        self.mode, self.limit, self.dim = mode, limit, dim
        self.index = IndexBinaryIDMap2(dim)
        self.store = {}

    def add(self, ids, X):
        ids = [int(i) for i in ids]
        for e in ids:
            if e in self.store:
                self.remove(e)
        codes, q, mm = encode_batch(self.mode, X, self.limit)
        self.index.add_with_ids(codes, np.asarray(ids, np.int64))
        for j, e in enumerate(ids):
            self.store[e] = (None if q is None else q[j], None if mm is None else mm[j], np.asarray(X[j]))

    def remove(self, e):
        if int(e) in self.store:
            self.index.remove_ids(np.array([int(e)], np.int64))
            del self.store[int(e)]

    def search(self, qv, k: int = 10, binary_oversample: int = 10, compare_float32: bool = False):
        qb, _, _ = encode_batch(self.mode, np.asarray(qv).reshape(1, -1), self.limit)
        K = min(k * binary_oversample, self.index.ntotal)
        D, L = self.index.search(qb, K)
        hits = [(int(e), int(d)) for e, d in zip(L[0], D[0]) if e != -1]
        if self.mode == "bin16":
            hits.sort(key=lambda h: h[1])
            return [(e, float(d)) for e, d in hits[:k]]
        out = []
        for e, _ in hits:
            q, mm, f = self.store[e]
            if compare_float32:
                row = np.asarray(f, np.float32).reshape(1, -1)
            else:
                row = dequantize(self.mode, q.reshape(1, -1), None if mm is None else mm.reshape(1, 2), self.limit,
                                 self.dim)
            out.append((e, float(dequant_scores(np.asarray(qv, np.float32).reshape(1, -1), row)[0, 0])))
        out.sort(key=lambda h: h[1], reverse=True)
        return out[:k]


def rerank_results(cand_ids, cand_docs, results):
    """``CohereVectorDBInt8.search_rerank_cohere``'s last step (``CohereVectorDBInt8.py:329-338``):
    each rerank result's ``index`` points into the candidate list; ``score`` = ``relevance_score``;
    Python's stable sort by score descending over the service's result order."""
    out = [{"doc_id": cand_ids[r["index"]], "score": r["relevance_score"], "doc": cand_docs[r["index"]]}
           for r in results]
    out.sort(key=lambda x: x["score"], reverse=True)
    return out
