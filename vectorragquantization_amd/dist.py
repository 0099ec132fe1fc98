"""Row-sharded three-phase search over several MI355X (one process per GPU).

The reference is single-process; sharding is this
build's only scaling axis.  Rank r owns a contiguous global row range
``[row0, row0 + m)`` (codes, int8 rows, norms, external ids).  A query batch is
replicated to every rank and searched in three steps:

1. local ``vrq_search3`` in ``VRQ_SEARCH_SHARD`` mode: the shard's exact top-K
   (K = the GLOBAL ``binary_k``, because the global top-K may sit in one shard)
   by (dist, global row), each with its Phase-II and Phase-III score;
2. ONE ``all_gather_into_tensor`` (RCCL over xGMI with the ``nccl`` backend) of
   the packed candidate tuples -- ``nq * K * 36`` bytes per rank (3.7 MB at
   nq = 1024, K = 100: latency-bound, one collective per batch);
3. ``vrq_merge_shards`` on every rank: global top-K by (dist, global row) ->
   stable sort by s2 -> first K3 -> stable sort by s3 -> first k, which is
   exactly the single-index semantics of ``CohereEnhancedVectorDB.py:267-322``,
   so results are identical for 1/2/4/8 ranks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _native as N
from .enhanced import SearchBatch, search3

# packed per-candidate record: row i64 | doc id i64 | s2 f64 | s3 f64 | dist i32  (36 B)
_REC = 36


def pack_candidates(count: torch.Tensor, rows: torch.Tensor, ids: torch.Tensor, dist_: torch.Tensor,
                    s2: torch.Tensor, s3: torch.Tensor) -> torch.Tensor:
    """Pack one rank's [nq, K] candidate tuples (+ counts) into a flat uint8 buffer."""
    nq, K = rows.shape
    parts = [count.to(torch.int32).contiguous().view(torch.uint8).reshape(-1),
             rows.contiguous().view(torch.uint8).reshape(-1),
             ids.contiguous().view(torch.uint8).reshape(-1),
             s2.contiguous().view(torch.uint8).reshape(-1),
             s3.contiguous().view(torch.uint8).reshape(-1),
             dist_.to(torch.int32).contiguous().view(torch.uint8).reshape(-1)]
    return torch.cat(parts)


def unpack_candidates(buf: torch.Tensor, S: int, nq: int, K: int):
    """Inverse of ``pack_candidates`` for S stacked ranks -> [S, nq(, K)] views."""
    b = buf.reshape(S, -1)
    o = 0

    def take(nbytes, dtype, shape):
        nonlocal o
        t = b[:, o:o + nbytes].contiguous().view(dtype).reshape(S, *shape)
        o += nbytes
        return t

    cnt = take(4 * nq, torch.int32, (nq,))
    rows = take(8 * nq * K, torch.int64, (nq, K))
    ids = take(8 * nq * K, torch.int64, (nq, K))
    s2 = take(8 * nq * K, torch.float64, (nq, K))
    s3 = take(8 * nq * K, torch.float64, (nq, K))
    d = take(4 * nq * K, torch.int32, (nq, K))
    return cnt, rows, ids, d, s2, s3


def gather_candidates(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather the packed buffers of every rank (single collective).  With the ``nccl`` backend
    (RCCL) device buffers travel GPU to GPU; a ``gloo`` group (CPU tests, several ranks sharing one
    GPU) stages the device buffer through host memory."""
    world = dist.get_world_size(group)
    stage = local.is_cuda and dist.get_backend(group) == "gloo"
    src = local.cpu() if stage else local
    out = torch.empty((world * src.numel(),), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out.to(local.device) if stage else out


def merge_shards(cnt, rows, d, s2, s3, k: int, K3: int):
    """``vrq_merge_shards`` on stacked [S, nq, K] tensors -> (count, rows, dist, s2, s3, src)."""
    S, nq, K = rows.shape
    dev = rows.device
    oc = torch.empty((nq,), dtype=torch.int32, device=dev)
    orow = torch.empty((nq, k), dtype=torch.int64, device=dev)
    od = torch.empty((nq, k), dtype=torch.int32, device=dev)
    o2 = torch.empty((nq, k), dtype=torch.float64, device=dev)
    o3 = torch.empty((nq, k), dtype=torch.float64, device=dev)
    src = torch.empty((nq, k), dtype=torch.int32, device=dev)
    cnt, rows, d, s2, s3 = (t.contiguous() for t in (cnt, rows, d, s2, s3))  # held until the launch returns
    lib = N.load()
    with torch.cuda.device(dev):
        rc = lib.vrq_merge_shards(S, nq, K, N.ptr(cnt), N.ptr(rows), N.ptr(d), N.ptr(s2), N.ptr(s3), k, K3,
                                  N.ptr(oc), N.ptr(orow), N.ptr(od), N.ptr(o2), N.ptr(o3), N.ptr(src),
                                  N.stream_handle(dev))
    N.check(rc, "vrq_merge_shards")
    return oc, orow, od, o2, o3, src


def merge_topk_shards(rows: torch.Tensor, scores: torch.Tensor, k: int):
    """Merge of row-sharded ``vrq_gemm_topk`` outputs (config 5) after the all-gather.

    ``rows``/``scores`` are [S, nq, k] (global rows; -1 / NaN padding).  Result: (count, rows,
    scores) of the global top-k in the reference's (score desc, row asc) order, identical to one
    call over the whole corpus.  Two stable sorts: by row (padding last), then by score descending
    (-0.0 equal to +0.0 and padding equal to -inf, both as in Python's sort; padding stays behind
    real -inf rows because it is last in row order)."""
    S, nq, kk = rows.shape
    r = rows.permute(1, 0, 2).reshape(nq, S * kk)
    sc = scores.permute(1, 0, 2).reshape(nq, S * kk)
    o = torch.sort(torch.where(r >= 0, r, torch.full_like(r, torch.iinfo(torch.int64).max)), dim=1,
                   stable=True).indices
    r, sc = torch.gather(r, 1, o), torch.gather(sc, 1, o)
    key = torch.where(r >= 0, sc, torch.full_like(sc, float("-inf"))) + 0.0  # + 0.0 maps -0.0 to +0.0
    o = torch.sort(-key, dim=1, stable=True).indices[:, :k]
    r, sc = torch.gather(r, 1, o), torch.gather(sc, 1, o)
    return (r >= 0).sum(1).to(torch.int32), r, sc


def gather_topk(rows: torch.Tensor, scores: torch.Tensor, group=None):
    """One all-gather of a rank's [nq, k] (rows i64, scores f64) -> stacked [S, nq, k] each."""
    S = dist.get_world_size(group)
    buf = torch.cat([rows.contiguous().view(torch.uint8).reshape(-1), scores.contiguous().view(torch.uint8).reshape(-1)])
    out = gather_candidates(buf, group).reshape(S, -1)
    h = rows.numel() * 8
    return (out[:, :h].contiguous().view(torch.int64).reshape(S, *rows.shape),
            out[:, h:].contiguous().view(torch.float64).reshape(S, *scores.shape))


class ShardedSearch:
    """One rank's shard of a row-sharded corpus + the collective search."""

    def __init__(self, codes: torch.Tensor, x8: torch.Tensor, norms: torch.Tensor, ids: torch.Tensor,
                 row0: int, n_total: int, group=None):
        self.codes, self.x8, self.norms, self.ids = codes, x8, norms, ids
        self.row0, self.n_total, self.group = int(row0), int(n_total), group
        self.device = codes.device
        self._ws = None

    def local(self, qf, qb, k, binary_oversample, int8_oversample):
        K = min(k * binary_oversample, self.n_total)
        lib = N.load()
        need = lib.vrq_search3_workspace_size(self.codes.shape[0], qf.shape[1], qf.shape[0], K) \
            if self.codes.shape[0] and K else 0
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty((max(need, 8),), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            cnt, rows, d, s2, s3 = search3(self.codes, self.x8, self.norms, qf, qb, k, K,
                                           k * int8_oversample, N.VRQ_SEARCH_SHARD, self.row0, None, self._ws)
        loc = (rows - self.row0).clamp_min(0)
        ids = torch.where(rows >= 0, self.ids[loc] if self.ids.numel() else rows, rows)
        return K, cnt, rows, ids, d, s2, s3

    def search_vectors(self, qf, qb, k: int = 10, binary_oversample: int = 10,
                       int8_oversample: int = 3) -> SearchBatch:
        K, cnt, rows, ids, d, s2, s3 = self.local(qf, qb, k, binary_oversample, int8_oversample)
        nq = qf.shape[0]
        S = dist.get_world_size(self.group)
        allb = gather_candidates(pack_candidates(cnt, rows, ids, d, s2, s3), self.group)
        gc, gr, gi, gd, g2, g3 = unpack_candidates(allb, S, nq, K)
        oc, orow, od, o2, o3, src = merge_shards(gc, gr, gd, g2, g3, k, k * int8_oversample)
        flat_ids = gi.permute(1, 0, 2).reshape(nq, S * K)  # [nq, S*K] in (shard, pos) order
        oid = torch.where(src >= 0, torch.gather(flat_ids, 1, src.clamp_min(0).to(torch.int64)),
                          torch.full_like(orow, -1))
        return SearchBatch(oc, oid, orow, od, o2, o3)
