import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvrq.so on cuda:0)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np
    return {name: np.load(os.path.join(GOLDEN, f"{name}.npz"))
            for name in ("encoders", "search_synth", "search_real", "dequant", "flat_real")}


@pytest.fixture(scope="session")
def oracle_lib():
    """ctypes handle of the C restatement of FAISS hammings_knn_hc (test infrastructure)."""
    import ctypes as C
    import subprocess
    so = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.check_call([os.path.join(REPO, "oracle", "build.sh")])
    lib = C.CDLL(so)
    lib.oracle_hamming_knn.restype = C.c_int
    lib.oracle_hamming_knn.argtypes = [C.c_void_p, C.c_int64, C.c_int, C.c_void_p, C.c_int, C.c_int,
                                       C.c_void_p, C.c_void_p, C.c_int]
    return lib


def oracle_knn(lib, codes, queries, k, threads=0):
    import numpy as np
    codes = np.ascontiguousarray(codes, dtype=np.uint8)
    queries = np.ascontiguousarray(queries, dtype=np.uint8)
    nq = queries.shape[0]
    D = np.empty((nq, k), np.int32)
    I = np.empty((nq, k), np.int64)
    rc = lib.oracle_hamming_knn(codes.ctypes.data, codes.shape[0], codes.shape[1], queries.ctypes.data, nq, k,
                                D.ctypes.data, I.ctypes.data, threads)
    assert rc == 0
    return D, I


@pytest.fixture(scope="session")
def golden_vdb():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "vectordb_synth.npz")))


@pytest.fixture(scope="session")
def golden_vdb_real():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "vectordb_real.npz")))


@pytest.fixture(scope="session")
def golden_cohere_int8():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "cohere_int8.npz")))
