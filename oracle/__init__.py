"""CPU oracle for the vectorragquantization_amd hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import, call, link or execute it, and only as the *checker* (or as the
timed CPU baseline), never as the thing measured or shipped.  The product path
(``vectorragquantization_amd``) never imports this package and fails loudly when
its HIP library is missing.

Contents
--------
* ``oracle_np``   -- NumPy restatement of the reference algorithm
  (``CohereEnhancedVectorDB.search`` Phases I-III, FAISS ``IndexBinaryFlat`` /
  ``IndexBinaryIDMap2`` semantics, the six ``VectorDBInt*`` encoders).
* ``hamming_knn.c`` -- plain-C restatement of FAISS ``hammings_knn_hc`` (heap
  top-k, strict ``<`` insert, OpenMP over queries) used as the timed CPU
  baseline for Phase I; built into ``oracle/_build/liboracle.so`` by
  ``oracle/build.sh`` (called from ``__graft_entry__.build()``).

Parity pinning: the encoders and Phases II/III are pinned against golden
vectors produced by the reference's *own* Python code (``tests/golden/
make_golden.py``, run in the survey container with FAISS/rocksdict stubbed).
Phase I lives in FAISS C++, which is absent from the reference tree and from
this image; its tie order is pinned only by the restated FAISS semantics
("parity unpinned" at the FAISS boundary -- see DESIGN.md section 3).
"""
