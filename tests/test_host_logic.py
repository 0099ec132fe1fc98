"""Host-side logic that needs no GPU: FAISS IBM2 on-disk format, providers, plans."""
import hashlib
import json

import numpy as np
import pytest

from vectorragquantization_amd.embed import CohereHTTPProvider, SyntheticCohereProvider, text_seed
from vectorragquantization_amd.index import ibm2_pack, ibm2_unpack


def test_ibm2_pack_reproduces_reference_index_bin(golden):
    g = golden["search_real"]
    b = ibm2_pack(1024, g["codes"], np.arange(1000, dtype=np.int64))
    assert len(b) == 136066
    assert hashlib.sha256(b).digest() == g["index_bin_sha256"].tobytes()
    d, xb, ids = ibm2_unpack(b)
    assert d == 1024 and np.array_equal(xb, g["codes"]) and np.array_equal(ids, np.arange(1000))


def test_ibm2_empty_and_bad_magic():
    b = ibm2_pack(1024, np.zeros((0, 128), np.uint8), np.zeros((0,), np.int64))
    d, xb, ids = ibm2_unpack(b)
    assert d == 1024 and xb.shape == (0, 128) and ids.shape == (0,)
    with pytest.raises(ValueError):
        ibm2_unpack(b"XXXX" + b[4:])


def test_synthetic_provider_is_deterministic_and_unit_norm():
    p = SyntheticCohereProvider()
    a = p.float_embeddings(["alpha", "beta"])
    b = p.float_embeddings(["alpha", "beta"])
    assert np.array_equal(a, b)
    assert np.allclose(np.linalg.norm(a, axis=1), 1.0, atol=1e-6)
    assert text_seed("alpha") == text_seed("alpha") != text_seed("beta")


def test_http_provider_requires_env_like_reference(monkeypatch):
    monkeypatch.delenv("COHERE_EMBED_ENDPOINT", raising=False)
    monkeypatch.delenv("COHERE_EMBED_KEY", raising=False)
    with pytest.raises(Exception, match="COHERE_EMBED_ENDPOINT"):
        CohereHTTPProvider()
    monkeypatch.setenv("COHERE_EMBED_ENDPOINT", "http://127.0.0.1:9")
    with pytest.raises(Exception, match="COHERE_EMBED_KEY"):
        CohereHTTPProvider()
    monkeypatch.setenv("COHERE_EMBED_KEY", "k")
    p = CohereHTTPProvider()
    assert p.endpoint.endswith("/v2/embed")
    # no network: failures are logged and {} returned, as in CohereEnhancedVectorDB.py:167-169
    assert p.embed(["x"], "search_query", ["float"]) == {}


def test_ixmp_pack_reproduces_reference_index_faiss(golden):
    """FloatIndexIDMap's writer: the reference's db_cohere_float/index.faiss byte-for-byte (its
    sha256 is in the fixture), and the reader inverts it."""
    from vectorragquantization_amd.flat import ixmp_pack, ixmp_unpack
    g = golden["flat_real"]
    b = ixmp_pack(1024, g["xf"], np.arange(1000))
    assert hashlib.sha256(b).digest() == g["index_faiss_sha256"].tobytes()
    d, xf, ids = ixmp_unpack(b)
    assert d == 1024 and np.array_equal(xf, g["xf"]) and np.array_equal(ids, np.arange(1000))
    with pytest.raises(ValueError):
        ixmp_unpack(b"IBM2" + b[4:])
    e = ixmp_pack(1024, np.zeros((0, 1024), np.float32), np.zeros(0, np.int64))
    d, xf, ids = ixmp_unpack(e)
    assert xf.shape == (0, 1024) and ids.shape == (0,)
