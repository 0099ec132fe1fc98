"""BASELINE config 4 at full size on one GPU, the RCCL leg, and opening the reference's own DB folders.

* 100M x 1024 corpus (SURVEY.md 8(d) generator) at the bench's batch of nq = 1024 (the MB = 4
  matrix-core kernel the headline number runs): the three-phase search of one index equals, bit for
  bit, the VRQ_SEARCH_SHARD searches of the 8 row ranges an 8-GPU run would own, merged by
  vrq_merge_shards (the multi-GPU semantics of CohereEnhancedVectorDB.py:267-322); the single index's
  Phase I equals the FAISS hammings_knn_hc restatement and its final rows and Phase-II scores equal the
  reference NumPy Phases II/III on 16 queries spread over both 512-query blocks (rows and Phase-II
  scores bit for bit, Phase-III cosines within 1e-5 relative).
* The same equality for 8 row ranges of 500K rows, each short enough (n * nq <= 2^32) to run K1s.
* ShardedSearch through a real ``nccl`` (RCCL) process group.
* ``CohereEnhancedVectorDB`` / ``CohereVectorDBFloat`` opening byte copies of the reference's persisted
  folders (tests/golden/ref_db: FAISS index + RocksDB tables) and reproducing its search output.
"""
import os
import shutil

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN, oracle_knn

pytestmark = pytest.mark.gpu

N100M = 100_000_000


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _phase23_reference(qf, codes_rows, x8_rows, rows, k=10, osi=3):
    """The reference's Phase II / III per query (CohereEnhancedVectorDB.py:281-322) on candidate rows."""
    pm = 2 * np.unpackbits(codes_rows, axis=1).astype(np.int32) - 1
    s2 = np.array([float(qf.dot(p)) for p in pm])
    o2 = sorted(range(len(rows)), key=lambda j: -s2[j])[: k * osi]
    s3 = []
    for j in o2:
        nrm = np.linalg.norm(x8_rows[j])
        s3.append(-np.inf if nrm == 0 else float(qf.dot(x8_rows[j])) / nrm)
    o3 = sorted(range(len(o2)), key=lambda j: -s3[j])[:k]
    return (np.array([rows[o2[j]] for j in o3], dtype=np.int64), np.array([s2[o2[j]] for j in o3]),
            np.array([s3[j] for j in o3]))


def test_100m_row_ranges_merge_equal_single_index(dev, oracle_lib):
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd import synth
    from vectorragquantization_amd.dist import merge_shards
    from vectorragquantization_amd.enhanced import search3

    nq, k = 1024, 10                         # the bench's batch: K1m with 4 M-blocks per wave (2 query blocks)
    sh = synth.make_corpus(N100M, device=dev)
    codes, x8, norms = sh["codes"], sh["x8"], sh["norms"]
    qf, qb, _ = synth.make_queries(N100M, nq, device=dev)
    full = [t.cpu().numpy() for t in search3(codes, x8, norms, qf, qb, k, 100, 30)]
    p1 = [t.cpu().numpy() for t in search3(codes, x8, norms, qf, qb, k, 100, 30, N.VRQ_SEARCH_PHASE1_ONLY)]
    parts = []
    for g in range(8):
        r0, r1 = synth.shard_range(N100M, g, 8)
        parts.append(search3(codes[r0:r1], x8[r0:r1], norms[r0:r1], qf, qb, k, 100, 30, N.VRQ_SEARCH_SHARD, r0))
    st = [torch.stack([p[i] for p in parts]) for i in range(5)]
    merged = [t.cpu().numpy() for t in merge_shards(st[0], st[1], st[2], st[3], st[4], k, 30)[:5]]
    for a, b in zip(merged, full):
        assert np.array_equal(a, b), "8 merged row ranges differ from the single 100M index"
    assert (full[0] == k).all()
    info = np.zeros(12, np.int64)
    N.check(N.load().vrq_scan_plan(N100M, 1024, nq, 100, 0, info.ctypes.data), "plan")
    assert (int(info[0]), int(info[1])) == (0, 4)          # K1m, MB = 4: the instance the bench times
    # Phase I of the single index vs the FAISS restatement, and the final rows vs the reference NumPy
    # Phases II/III on those candidates, for 16 queries spread over both 512-query blocks
    qsel = np.linspace(0, nq - 1, 16).round().astype(np.int64)
    assert (qsel < 512).any() and (qsel >= 512).any()
    codes_h = codes.cpu().numpy()
    D, I = oracle_knn(oracle_lib, codes_h, qb[torch.from_numpy(qsel).to(dev)].cpu().numpy(), 100, threads=16)
    assert np.array_equal(p1[2][qsel], D) and np.array_equal(p1[1][qsel], I)
    qf_h = qf.cpu().numpy()
    for i, q in enumerate(qsel):
        rows = I[i]
        x8r = x8[torch.from_numpy(rows).to(dev)].cpu().numpy()
        ref_rows, ref_s2, ref_s3 = _phase23_reference(qf_h[q], codes_h[rows], x8r, rows)
        assert np.array_equal(full[1][q], ref_rows)
        assert np.array_equal(full[3][q], ref_s2)
        # Phase III: exact f64 dot rounded once vs NumPy's f32 sdot, within 1e-5 relative
        np.testing.assert_allclose(full[4][q], ref_s3, rtol=1e-5, atol=1e-7)
    del codes_h, sh, codes, x8, norms
    torch.cuda.empty_cache()


def test_k1s_row_ranges_merge_equal_single_index(dev, oracle_lib):
    """8 row ranges of 500K rows at nq = 1024 (per-shard n * nq <= 2^32: every shard runs K1s, as
    config 2 does at N = 8), merged by vrq_merge_shards, equal the single 4M-row index bit for bit."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd import synth
    from vectorragquantization_amd.dist import merge_shards
    from vectorragquantization_amd.enhanced import search3

    n, nq, k = 4_000_000, 1024, 10
    sh = synth.make_corpus(n, device=dev)
    codes, x8, norms = sh["codes"], sh["x8"], sh["norms"]
    qf, qb, _ = synth.make_queries(n, nq, device=dev)
    full = [t.cpu().numpy() for t in search3(codes, x8, norms, qf, qb, k, 100, 30)]
    info = np.zeros(12, np.int64)
    parts = []
    for g in range(8):
        r0, r1 = synth.shard_range(n, g, 8)
        N.check(N.load().vrq_scan_plan(r1 - r0, 1024, nq, 100, 0, info.ctypes.data), "plan")
        assert int(info[0]) == 2, "shard does not run K1s"
        parts.append(search3(codes[r0:r1], x8[r0:r1], norms[r0:r1], qf, qb, k, 100, 30, N.VRQ_SEARCH_SHARD, r0))
    st = [torch.stack([p[i] for p in parts]) for i in range(5)]
    merged = [t.cpu().numpy() for t in merge_shards(st[0], st[1], st[2], st[3], st[4], k, 30)[:5]]
    for a, b in zip(merged, full):
        assert np.array_equal(a, b), "8 merged K1s row ranges differ from the single index"
    assert (full[0] == k).all()
    # the single index's Phase I (K1s at 4M x 1024) vs the FAISS restatement on a query sample
    qsel = np.linspace(0, nq - 1, 32).round().astype(np.int64)
    p1 = [t.cpu().numpy() for t in search3(codes, x8, norms, qf, qb, k, 100, 30, N.VRQ_SEARCH_PHASE1_ONLY)]
    D, I = oracle_knn(oracle_lib, codes.cpu().numpy(), qb[torch.from_numpy(qsel).to(dev)].cpu().numpy(), 100,
                      threads=16)
    assert np.array_equal(p1[2][qsel], D) and np.array_equal(p1[1][qsel], I)
    del sh, codes, x8, norms
    torch.cuda.empty_cache()


def test_sharded_search_through_nccl(dev):
    """ShardedSearch's all-gather + merge over a real RCCL process group (world 1 on the one GPU of the
    box; the driver's 8-GPU run uses the same code with 8 ranks) equals the single-index search."""
    import socket

    import torch.distributed as dist

    from vectorragquantization_amd.dist import ShardedSearch
    from vectorragquantization_amd.enhanced import search3
    from vectorragquantization_amd.quant import encode, int8_row_norms

    rng = np.random.default_rng(5)
    n, nq = 200_000, 160
    F = torch.from_numpy(rng.standard_normal((n, 1024)).astype(np.float32) * 0.03).to(dev)
    e = encode("cohere", F, 0.1, dev)
    codes, x8 = e["codes"], e["q"]
    norms = int8_row_norms(x8)
    qf = F[torch.from_numpy(rng.integers(0, n, nq)).to(dev)] + 0.01 * torch.randn((nq, 1024), device=dev)
    qb = encode("cohere", qf, 0.1, dev)["codes"]
    ids = torch.arange(n, dtype=torch.int64, device=dev) * 3 + 7
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        res = ShardedSearch(codes, x8, norms, ids, 0, n).search_vectors(qf, qb, 10, 10, 3)
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    cnt, rows, d, s2, s3 = search3(codes, x8, norms, qf, qb, 10, 100, 30)
    assert torch.equal(res.count, cnt) and torch.equal(res.row, rows) and torch.equal(res.hamming, d)
    assert torch.equal(res.binary, s2) and torch.equal(res.cosine, s3)
    assert torch.equal(res.doc_id, torch.where(rows >= 0, ids[rows.clamp_min(0)], rows))


class _Lookup:
    """Embedding provider replaying the golden query embeddings (the reference's HTTP call replaced)."""

    def __init__(self, table):
        self.table = table

    def embed(self, texts, input_type, embedding_types):
        fl, ub = zip(*(self.table[t] for t in texts))
        out = {"float": np.stack(fl)}
        if "ubinary" in embedding_types:
            out["ubinary"] = np.stack(ub)
        return out


def test_open_reference_enhanced_folder(tmp_path, dev, golden):
    """CohereEnhancedVectorDB(<copy of the reference's db_cohere_enhanced>) loads its FAISS index.bin and
    all 1000 documents from its RocksDB docs/ and returns exactly the reference's own search() output."""
    from vectorragquantization_amd.enhanced import CohereEnhancedVectorDB
    src = os.path.join(GOLDEN, "ref_db", "db_cohere_enhanced")
    dst = tmp_path / "db_cohere_enhanced"
    shutil.copytree(src, dst)
    g = golden["search_real"]
    prov = _Lookup({f"q{i}": (g["qf"][i], g["qb"][i]) for i in range(g["qf"].shape[0])})
    db = CohereEnhancedVectorDB(str(dst), provider=prov, device=dev)
    assert len(db) == 1000 and len(db.texts) == 1000
    for i in range(0, g["qf"].shape[0], 7):
        res = db.search(f"q{i}", k=10)
        n = int(g["k10_cnt"][i])
        assert [h["doc_id"] for h in res] == g["k10_ids"][i][:n].tolist()
        assert [h["score_hamming"] for h in res] == g["k10_ham"][i][:n].tolist()
        assert [h["score_binary"] for h in res] == g["k10_bin"][i][:n].tolist()
        np.testing.assert_allclose([h["score_cosine"] for h in res], g["k10_cos"][i][:n], rtol=1e-5)
        assert all(h["doc"] == db.texts[h["doc_id"]] and h["doc"] != "N/A" for h in res)
    # batch surface: the whole query table at once
    b = db.search_vectors(g["qf"], g["qb"], 10, 10, 3)
    assert np.array_equal(b.doc_id.cpu().numpy(), g["k10_ids"])
    # remove + save writes this build's store beside the RocksDB directory, which stays untouched
    before = sorted(os.listdir(dst / "docs"))
    db.remove_document(3, save=True)
    assert sorted(os.listdir(dst / "docs")) == before
    db2 = CohereEnhancedVectorDB(str(dst), provider=prov, device=dev)
    assert len(db2) == 999 and 3 not in db2.texts
    assert db2.search("q0", k=10) == db.search("q0", k=10)


def test_open_reference_float_folder(tmp_path, dev, golden):
    """CohereVectorDBFloat on the reference's db_cohere_float folder (its RocksDB texts + an index.faiss
    written from the persisted floats, byte-identical to the reference's file)."""
    import hashlib

    from vectorragquantization_amd.flat import CohereVectorDBFloat, ixmp_pack
    g = golden["flat_real"]
    dst = tmp_path / "db_cohere_float"
    shutil.copytree(os.path.join(GOLDEN, "ref_db", "db_cohere_float"), dst)
    img = ixmp_pack(1024, g["xf"], np.arange(1000, dtype=np.int64))
    assert hashlib.sha256(img).digest() == bytes(g["index_faiss_sha256"])
    (dst / "index.faiss").write_bytes(img)
    prov = _Lookup({})
    db = CohereVectorDBFloat(str(dst), provider=prov, device=dev)
    assert len(db) == 1000 and len(db.texts) == 1000
    from oracle import oracle_np as O
    q = g["qf"]
    cnt, ids, sc = db.search_vectors(torch.from_numpy(q).to(dev), 10)
    ref_sc, ref_rows = O.flat_ip_search(g["xf"], q, 10)
    assert np.array_equal(ids.cpu().numpy(), ref_rows)        # ids = rows: the folder holds ids 0..999 in order
    assert np.array_equal(sc.cpu().numpy(), ref_sc)
    prov.table["x"] = (q[3], None)
    hits = db.search("x", k=5)
    assert [h["doc_id"] for h in hits] == ref_rows[3][:5].tolist()
    assert all(h["doc"] == db.texts[h["doc_id"]] and h["doc"] != "N/A" for h in hits)


def test_inconsistent_store_is_refused(tmp_path, dev):
    """An index whose int8 store is short is refused before any launch (the ABI cannot see x8's length)."""
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.embed import SyntheticCohereProvider
    from vectorragquantization_amd.enhanced import CohereEnhancedVectorDB
    from vectorragquantization_amd.docstore import DocStoreError
    prov = SyntheticCohereProvider(device=dev)
    db = CohereEnhancedVectorDB(str(tmp_path / "db"), provider=prov, device=dev)
    db.add_documents(list(range(50)), [f"doc {i}" for i in range(50)], save=True)
    db._x8.n -= 1                                           # the state a missing doc store used to leave
    with pytest.raises(N.VrqNativeError):
        db.search("doc 3", k=5)
    shutil.rmtree(tmp_path / "db" / "vrq_docs")             # index.bin without any document store
    with pytest.raises(DocStoreError):
        CohereEnhancedVectorDB(str(tmp_path / "db"), provider=prov, device=dev)
