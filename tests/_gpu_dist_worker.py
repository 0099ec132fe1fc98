"""One rank of tests/test_gpu_dist.py: the product's row-sharded search across real processes.

Started by the test as a child process with WORLD_SIZE / RANK / MASTER_* set; every rank shares
cuda:0 of the one-GPU box and the ``gloo`` group stages the packed candidates through host memory
(the 8-GPU driver run uses the same code over ``nccl``).  Each rank builds only its row shard of the
synthetic corpus (SURVEY.md 8(d) generator) and runs the library on it:

* config 4: ``ShardedSearch.search_vectors`` = ``vrq_search3(..., VRQ_SEARCH_SHARD)`` on the shard ->
  ``pack_candidates`` -> one all-gather -> ``unpack_candidates`` -> ``vrq_merge_shards``, for a
  K1m-sized batch (nq = 256) and a K1r-sized one (nq = 64);
* config 5: ``vrq_gemm_topk`` (both phases) on the shard with its global row offset ->
  ``gather_topk`` -> ``merge_topk_shards``.

Rank 0 then builds the whole corpus and checks every merged tensor equal to the single-index call
(``CohereEnhancedVectorDB.py:267-322`` semantics; ``:283-293`` / ``:302-318`` for config 5).  It
writes ``OK`` or the first mismatch to $VRQ_DIST_RESULT and exits non-zero on a mismatch."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from vectorragquantization_amd import _native as N  # noqa: E402
from vectorragquantization_amd import synth  # noqa: E402
from vectorragquantization_amd.dist import ShardedSearch, gather_topk, merge_topk_shards  # noqa: E402
from vectorragquantization_amd.enhanced import gemm_topk, search3  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    n = int(os.environ.get("VRQ_DIST_ROWS", "1000000"))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    N.load()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = synth.make_corpus(n, rank=rank, world=world, device=dev)
    codes, x8, norms, row0 = sh["codes"], sh["x8"], sh["norms"], sh["row0"]
    ids = torch.arange(row0, row0 + codes.shape[0], dtype=torch.int64, device=dev) * 3 + 11  # external ids
    k = 10
    got = {}
    for nq in (256, 64):
        qf, qb, _ = synth.make_queries(n, nq, device=dev)
        res = ShardedSearch(codes, x8, norms, ids, row0, n).search_vectors(qf, qb, k, 10, 3)
        got[("c4", nq)] = (res.count, res.row, res.hamming, res.binary, res.cosine, res.doc_id)
    qf5, _, _ = synth.make_queries(n, 256, device=dev)
    for mode in ("binary", "int8_cosine"):
        _, r, s = gemm_topk(mode, qf5, k, codes=codes, x8=x8, norms=norms, row_offset=row0)
        gr, gs = gather_topk(r, s)
        got[("c5", mode)] = merge_topk_shards(gr, gs, k)
    torch.cuda.synchronize()
    dist.barrier()
    msg = "OK"
    if rank == 0:
        del codes, x8, norms, sh
        full = synth.make_corpus(n, device=dev)
        fc, fx, fn = full["codes"], full["x8"], full["norms"]
        fids = torch.arange(n, dtype=torch.int64, device=dev) * 3 + 11
        names = ("count", "row", "hamming", "binary", "cosine", "doc_id")
        for nq in (256, 64):
            qf, qb, _ = synth.make_queries(n, nq, device=dev)
            c, r, d, s2, s3 = search3(fc, fx, fn, qf, qb, k, 10 * k, 3 * k)
            ref = (c, r, d, s2, s3, torch.where(r >= 0, fids[r.clamp_min(0)], r))
            for nm, a, b in zip(names, got[("c4", nq)], ref):
                if not torch.equal(a, b):
                    msg = f"config 4 nq={nq}: merged {nm} differs from the single index"
                    break
            if msg != "OK":
                break
            if not bool((c == k).all()):
                msg = f"config 4 nq={nq}: short result"
        for mode in ("binary", "int8_cosine"):
            if msg != "OK":
                break
            ref = gemm_topk(mode, qf5, k, codes=fc, x8=fx, norms=fn)
            for nm, a, b in zip(("count", "rows", "scores"), got[("c5", mode)], ref):
                if not torch.equal(a, b):
                    msg = f"config 5 {mode}: merged {nm} differs from the single corpus"
                    break
        with open(os.environ["VRQ_DIST_RESULT"], "w") as f:
            f.write(msg)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if msg == "OK" else 1)


if __name__ == "__main__":
    main()
