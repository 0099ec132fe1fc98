"""GPU parity of the VectorDB* search side: device dequantisation against the
reference's own `_dequantize_*` (golden, bit-exact), the dequantised-dot rescoring against the
reference's `float(np.dot(query_float, doc_emb))` (golden, float32-dot tolerance), and the whole
search (Phase I Hamming top-K -> rescoring -> stable sort -> k) against the oracle restatement."""
import numpy as np
import pytest
import torch

from oracle import oracle_np as O
from tests.test_oracle_golden import DEQ_KEYS, deq_inputs, score_close

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from vectorragquantization_amd import _native
    _native.load()
    return torch.device("cuda", 0)


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("key", DEQ_KEYS)
def test_dequantize_bit_exact_vs_reference_golden(golden, dev, key):
    from vectorragquantization_amd.quant import dequantize
    E, G = golden["encoders"], golden["dequant"]
    mode, q, mm, lim = deq_inputs(E, key)
    got = dequantize(mode, q, minmax=mm, limit=lim, dim=1024, device=dev).cpu().numpy()
    assert np.array_equal(got, G[key]), key


@pytest.mark.parametrize("key", DEQ_KEYS)
def test_rescore_dequant_vs_reference_golden(golden, dev, key):
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.quant import _DEQ_MODES
    E, G = golden["encoders"], golden["dequant"]
    mode, q, mm, lim = deq_inputs(E, key)
    n, nq = q.shape[0], G["qf"].shape[0]
    cand = np.tile(np.arange(-1, n, dtype=np.int64), (nq, 1))           # every row, plus a missing one
    q_t, qf_t, c_t = _t(q, dev), _t(G["qf"], dev), _t(cand, dev)
    mm_t = _t(mm, dev) if mm is not None else None
    out = torch.empty(cand.shape, dtype=torch.float64, device=dev)
    lib = N.load()
    N.check(lib.vrq_rescore_dequant(_DEQ_MODES[mode], N.ptr(qf_t), nq, 1024, N.ptr(q_t), N.ptr(mm_t), lim, n,
                                    N.ptr(c_t), cand.shape[1], N.ptr(out), N.stream_handle(dev)), "rescore")
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    assert np.all(np.isnan(o[:, 0]))
    S = O.dequant_scores(G["qf"], G[key])
    assert np.array_equal(o[:, 1:], S), key                               # the correctly rounded f32 dot
    for qi in range(nq):
        assert np.all(score_close(o[qi, 1:], G[f"score_{key}"][qi], G["qf"][qi], G[key]))


@pytest.mark.parametrize("mode", ["int8g", "int16g", "int4g", "int8", "int4", "bin16"])
def test_vectordb_search_vs_oracle(dev, mode):
    from vectorragquantization_amd.quant import encode, vectordb_search
    rng = np.random.default_rng(31)
    n, nq, k, osb, lim = 20_000, 24, 10, 10, 0.3
    C = rng.standard_normal((64, 1024)) / 32.0
    F = (C[rng.integers(0, 64, n)] + (0.6 / 32.0) * rng.standard_normal((n, 1024))).astype(np.float32)
    F[7] = F[3]                                                           # exact ties
    qf = (F[rng.integers(0, n, nq)] + 0.005 * rng.standard_normal((nq, 1024))).astype(np.float32)
    if mode == "bin16":
        X16 = np.clip(F * 30000, -32767, 32767).astype(np.int16)
        codes = encode("bin16", X16, device=dev)["codes"]
        qb = encode("bin16", np.clip(qf * 30000, -32767, 32767).astype(np.int16), device=dev)["codes"]
        rows, ham, sc = vectordb_search("bin16", codes, None, None, qb, k, osb)
        D, I = O.binary_flat_search(codes.cpu().numpy(), qb.cpu().numpy(), k)
        assert np.array_equal(rows.cpu().numpy(), I) and np.array_equal(ham.cpu().numpy(), D)
        return
    enc = encode(mode, F, lim, device=dev)
    qb = encode(mode, qf, lim, device=dev)["codes"]
    codes, q, mm = enc["codes"], enc["q"], enc["minmax"]
    qf_t = _t(qf, dev)
    rows, ham, sc = vectordb_search(mode, codes, q, qf_t, qb, k, osb, minmax=mm, limit=lim)
    rows, ham, sc = rows.cpu().numpy(), ham.cpu().numpy(), sc.cpu().numpy()
    # oracle: FAISS order Phase I, reference rescoring expression, Python stable sort
    D, I = O.binary_flat_search(codes.cpu().numpy(), qb.cpu().numpy(), min(k * osb, n))
    deq = O.dequantize(mode, q.cpu().numpy(), mm.cpu().numpy() if mm is not None else None, lim)
    for qi in range(nq):
        cand = I[qi][I[qi] >= 0]
        s = O.dequant_scores(qf[qi:qi + 1], deq[cand])[0]
        order = sorted(range(len(cand)), key=lambda j: -s[j])[:k]
        assert np.array_equal(rows[qi], cand[order]), (mode, qi)
        assert np.array_equal(sc[qi], s[order])
        assert np.array_equal(ham[qi], D[qi][order])
