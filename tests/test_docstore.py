"""The product's read-only RocksDict reader (vectorragquantization_amd/docstore.py) on the
reference's own persisted RocksDB tables (tests/golden/ref_db: byte copies of its data files),
plus the SST / WAL / Snappy / pickle decoding edge cases.  CPU only."""
import io
import os
import pickle
import struct

import numpy as np
import pytest

from conftest import GOLDEN
from vectorragquantization_amd import docstore as D

REF_DB = os.path.join(GOLDEN, "ref_db")


def test_reads_enhanced_docs_like_the_golden_walker(golden):
    """db_cohere_enhanced/docs: all 1000 {"doc", "int8"} records; the int8 rows equal the ones the
    fixture generator recovered independently (search_real.npz)."""
    r = D.RocksDictReader(os.path.join(REF_DB, "db_cohere_enhanced", "docs"))
    assert len(r) == 1000
    g = golden["search_real"]
    for i in range(1000):
        v = r[str(i)]
        assert set(v) == {"doc", "int8"}
        assert v["int8"].dtype == np.int8 and v["int8"].shape == (1024,)
        assert np.array_equal(v["int8"], g["int8"][i])
        assert isinstance(v["doc"], str) and v["doc"]


def test_snappy_compressed_table_and_float_store():
    """db_int4_global's SST is Snappy-compressed (only ~25 of its records are visible raw): every
    record decodes, and the texts equal the uncompressed enhanced DB's texts for the same ids (the
    reference built all its DBs from the same CSV rows)."""
    enh = D.RocksDictReader(os.path.join(REF_DB, "db_cohere_enhanced", "docs"))
    i4 = D.RocksDictReader(os.path.join(REF_DB, "db_int4_global", "docs"))
    fl = D.RocksDictReader(os.path.join(REF_DB, "db_cohere_float", "docs"))
    assert len(i4) == len(fl) == 1000
    for i in range(1000):
        a, b, c = enh[str(i)], i4[str(i)], fl[str(i)]
        assert b["doc"] == a["doc"] == c["doc"]
        assert b["emb_int4"].dtype == np.int8 and b["emb_int4"].shape == (512,)
        assert set(c) == {"doc"}


def test_snappy_literals_and_overlapping_copies():
    # "abcd" literal (tag (4-1) << 2), then a copy-1 element of length 8 ((8-4) << 2 | 1) at offset 4:
    # it overlaps its own output
    raw = bytes([12]) + bytes([3 << 2]) + b"abcd" + bytes([(8 - 4) << 2 | 1]) + bytes([4])
    # uncompressed length 12: "abcd" + 8 copied bytes "abcdabcd"
    assert D.snappy_decompress(raw) == b"abcdabcdabcd"
    # copy-2 element: tag (len-1)<<2 | 2, 16-bit offset
    raw2 = bytes([9]) + bytes([2 << 2]) + b"xyz" + bytes([(6 - 1) << 2 | 2]) + struct.pack("<H", 3)
    assert D.snappy_decompress(raw2) == b"xyzxyzxyz"
    with pytest.raises(D.DocStoreError):
        D.snappy_decompress(bytes([5]) + bytes([(4 - 1) << 2 | 2]) + struct.pack("<H", 1))


def _rd_key(s):
    return b"\x02" + s.encode()


def _rd_pickle(obj):
    return b"\x06" + pickle.dumps(obj, protocol=4)


def _wal_file(batches):
    """A RocksDB WAL: each WriteBatch in one FULL record (or FIRST/LAST when split over blocks)."""
    out = bytearray()
    for seq, ops in batches:
        w = bytearray(struct.pack("<QI", seq, len(ops)))
        for op in ops:
            if op[0] == "put":
                w += b"\x01" + bytes([len(op[1])]) + op[1]
                v = op[2]
                vl = bytearray()
                n = len(v)
                while n >= 0x80:
                    vl.append(n & 0x7F | 0x80)
                    n >>= 7
                vl.append(n)
                w += vl + v
            else:
                w += b"\x00" + bytes([len(op[1])]) + op[1]
        left = 32768 - len(out) % 32768
        if len(w) + 7 <= left:
            out += struct.pack("<IHB", 0, len(w), 1) + w
        else:  # FIRST fragment fills the block, LAST carries the rest
            a = left - 7
            out += struct.pack("<IHB", 0, a, 2) + w[:a]
            out += struct.pack("<IHB", 0, len(w) - a, 4) + w[a:]
    return bytes(out)


def test_wal_puts_deletes_and_sequence_order(tmp_path):
    big = np.arange(40000, dtype=np.int64) % 127
    x = np.arange(1024, dtype=np.int8)
    wal = _wal_file([
        (10, [("put", _rd_key("1"), _rd_pickle({"doc": "one", "int8": x})),
              ("put", _rd_key("2"), _rd_pickle({"doc": "two", "int8": x[::-1].copy()}))]),
        (12, [("del", _rd_key("1"))]),
        (13, [("put", _rd_key("2"), _rd_pickle({"doc": "two-v2", "int8": x})),
              ("put", _rd_key("3"), _rd_pickle({"doc": "big", "int8": big.astype(np.int8)}))]),  # spans blocks
    ])
    d = tmp_path / "docs"
    d.mkdir()
    (d / "000004.log").write_bytes(wal)
    r = D.RocksDictReader(str(d))
    assert sorted(r.keys()) == ["2", "3"]
    assert r["2"]["doc"] == "two-v2" and np.array_equal(r["2"]["int8"], x)
    assert np.array_equal(r["3"]["int8"], big.astype(np.int8))
    assert r.get("1") is None


def test_safe_unpickle_values_and_refusals():
    v = {"doc": "t", "emb_int16": np.arange(-5, 5, dtype="<i2"), "min_max": (np.float32(-0.5), np.float64(0.25)),
         "f": np.arange(6, dtype=np.float32).reshape(2, 3), "l": [1, 2.5, None, True]}
    out = D.safe_unpickle(pickle.dumps(v, protocol=4))
    assert out["doc"] == "t" and out["l"] == [1, 2.5, None, True]
    assert out["emb_int16"].dtype == np.dtype("<i2") and np.array_equal(out["emb_int16"], v["emb_int16"])
    assert out["min_max"] == (np.float32(-0.5), 0.25) and type(out["min_max"][0]) is np.float32
    assert np.array_equal(out["f"], v["f"])
    for bad in (pickle.dumps(print, protocol=4), pickle.dumps(io.BytesIO, protocol=2),
                pickle.dumps(np.array([{"a": 1}], dtype=object), protocol=4)):
        with pytest.raises(D.DocStoreError):
            D.safe_unpickle(bad)


def test_rocksdict_scalar_encodings():
    assert D.decode_rocksdict(b"\x02abc") == "abc"
    assert D.decode_rocksdict(b"\x01\x00\xff") == b"\x00\xff"
    # int / float payloads: byte order pinned by no reference artefact -> refused, never guessed
    for bad in (b"\x7f", b"\x03" + (-7).to_bytes(8, "little", signed=True), b"\x04" + struct.pack("<d", 1.5)):
        with pytest.raises(D.DocStoreError):
            D.decode_rocksdict(bad)


def _vi(n):
    out = bytearray()
    while n >= 0x80:
        out.append(n & 0x7F | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def test_write_batch_column_family_records():
    """RocksDB ValueType tags: 0x4 CF deletion, 0x5 CF value, 0x8 CF single deletion carry a family
    id; other families' records are consumed (their payload and sequence number) but not returned;
    LogData / Noop carry no sequence number; range deletions and merges are refused."""
    k, v = _rd_key("7"), _rd_pickle({"doc": "x"})
    rec = b"".join([
        b"\x05" + _vi(3) + _vi(len(k)) + k + _vi(len(v)) + v,   # CF 3 put of the same key: not ours
        b"\x03" + _vi(4) + b"blob",                              # LogData: no sequence number
        b"\x05" + _vi(0) + _vi(len(k)) + k + _vi(len(v)) + v,   # default-CF put via the CF form
        b"\x04" + _vi(3) + _vi(len(k)) + k,                      # CF 3 delete
        b"\x0d",                                                 # Noop
        b"\x08" + _vi(0) + _vi(len(k)) + k,                      # default-CF single deletion
        b"\x01" + _vi(len(k)) + k + _vi(len(v)) + v,            # plain put
    ])
    w = struct.pack("<QI", 100, 5) + rec
    out = list(D._write_batch(w))
    assert [(key, seq, typ) for key, seq, typ, _ in out] == [(k, 101, 1), (k, 103, 0), (k, 104, 1)]
    assert out[0][3] == v and out[2][3] == v
    for tag in (b"\x0f", b"\x0e" + _vi(0), b"\x02"):
        with pytest.raises(D.DocStoreError):
            list(D._write_batch(struct.pack("<QI", 1, 1) + tag + _vi(len(k)) + k + _vi(1) + b"z"))


def test_safe_unpickle_protocol5_arrays():
    x = np.arange(-6, 6, dtype=np.int8).reshape(3, 4)
    f = np.asfortranarray(np.arange(6, dtype="<f4").reshape(2, 3))
    out = D.safe_unpickle(pickle.dumps({"int8": x, "f": f, "doc": "d"}, protocol=5))
    assert np.array_equal(out["int8"], x) and out["int8"].dtype == np.int8
    assert np.array_equal(out["f"], f) and out["doc"] == "d"
    bufs = []
    with pytest.raises(D.DocStoreError):  # out-of-band buffers (NEXT_BUFFER) are refused
        D.safe_unpickle(pickle.dumps(x, protocol=5, buffer_callback=bufs.append))


def test_search3_refuses_inconsistent_rows():
    """The C ABI indexes x8 / norms by code row without their lengths; the wrapper refuses a short store
    before anything reaches the device (reference-folder opens used to leave it empty)."""
    import torch
    from vectorragquantization_amd import _native as N
    from vectorragquantization_amd.enhanced import search3
    codes = torch.zeros((10, 128), dtype=torch.uint8)
    qf, qb = torch.zeros((1, 1024)), torch.zeros((1, 128), dtype=torch.uint8)
    with pytest.raises(N.VrqNativeError):
        search3(codes, torch.zeros((0, 1024), dtype=torch.int8), torch.zeros((0,), dtype=torch.float64), qf, qb,
                10, 10, 10)
    with pytest.raises(N.VrqNativeError):
        search3(codes, torch.zeros((10, 1024), dtype=torch.int8), torch.zeros((9,), dtype=torch.float64), qf, qb,
                10, 10, 10)
