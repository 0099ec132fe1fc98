"""Read-only access to the reference's RocksDict document stores (``folder/docs``).

The reference keeps every document in a RocksDB database opened through rocksdict
(``Rdict(os.path.join(folder, "docs"))``, ``CohereEnhancedVectorDB.py:85-88``), one
entry per document: key ``str(doc_id)``, value ``{"doc": text, "int8": int8[1024]}``
(``:221``; the VectorDB* classes store ``emb_int8`` / ``emb_int16`` / ``emb_int4`` /
``min_max`` the same way).  Neither RocksDB nor rocksdict is a dependency of this
build, so opening a folder the reference wrote needs this reader:

* RocksDB block-based tables (``*.sst``, format_version 2..6, footer with or without the
  index handle, Snappy or uncompressed blocks, binary-search data blocks) and write-ahead
  logs (``*.log``: 32 KiB blocks of FULL/FIRST/MIDDLE/LAST records carrying WriteBatches).
  Entries are resolved by sequence number, deletions honoured.
* rocksdict's value encoding: one type byte (0x01 bytes, 0x02 str, 0x03 int, 0x04 float,
  0x05 bool, 0x06 pickle) before the payload; keys are encoded the same way.
* the pickles are decoded by a restricted interpreter of the pickle opcodes that executes
  nothing: it only builds dicts, lists, tuples, strings, numbers, bytes and NumPy arrays
  (``numpy.core.multiarray._reconstruct`` / ``scalar`` + ``numpy.ndarray`` + ``numpy.dtype``); any other
  global raises ``DocStoreError``.

Checksums are not verified.  Every ``*.sst`` file in the directory is read (RocksDB
deletes obsolete table files after compaction).
"""
from __future__ import annotations

import glob
import io
import logging
import os
import pickletools
import struct

import numpy as np

logger = logging.getLogger(__name__)


class DocStoreError(RuntimeError):
    pass


# --------------------------------------------------------------------------- varints / snappy
def _varint(b, p):
    r = s = 0
    while True:
        if p >= len(b):
            raise DocStoreError("truncated varint")
        c = b[p]
        p += 1
        r |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return r, p


def snappy_decompress(b: bytes) -> bytes:
    """Raw Snappy block format (the RocksDB kSnappyCompression payload)."""
    n, p = _varint(b, 0)
    out = bytearray()
    while p < len(b):
        tag = b[p]
        p += 1
        t = tag & 3
        if t == 0:  # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(b[p:p + nb], "little")
                p += nb
            ln += 1
            out += b[p:p + ln]
            p += ln
            continue
        if t == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | b[p]
            p += 1
        elif t == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(b[p:p + 2], "little")
            p += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(b[p:p + 4], "little")
            p += 4
        if off == 0 or off > len(out):
            raise DocStoreError("bad snappy copy offset")
        for _ in range(ln):  # byte-wise: copies may overlap their own output
            out.append(out[-off])
    if len(out) != n:
        raise DocStoreError("snappy length mismatch")
    return bytes(out)


# --------------------------------------------------------------------------- SST tables
_BLOCK_MAGIC = 0x88E241B785F4CFF7   # kBlockBasedTableMagicNumber
_LEGACY_MAGIC = 0xDB4775248B80FB57  # kLegacyBlockBasedTableMagicNumber
_TRAILER = 5                        # compression type + 32-bit checksum after every block


def _read_block(b: bytes, off: int, size: int) -> bytes:
    raw = b[off:off + size]
    ctype = b[off + size]
    if ctype == 0:
        return raw
    if ctype == 1:
        return snappy_decompress(raw)
    raise DocStoreError(f"unsupported block compression type {ctype}")


def _block_entries(blk: bytes, index_block: bool = False, delta_values: bool = False):
    """(key, value) pairs of a block.  Data/metaindex blocks: shared | unshared | value_len | key delta |
    value.  Index blocks with delta-encoded values (format_version >= 4): shared | unshared | key delta |
    BlockHandle (the value length is implied)."""
    nr_raw = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    if nr_raw & 0x80000000:
        raise DocStoreError("data blocks with a hash index are not supported")
    nres = nr_raw & 0x7FFFFFFF
    end = len(blk) - 4 - 4 * nres
    restarts = set(struct.unpack_from(f"<{nres}I", blk, end)) if nres else {0}
    p, key = 0, b""
    prev_off = prev_size = None
    while p < end:
        at_restart = p in restarts
        sh, p = _varint(blk, p)
        un, p = _varint(blk, p)
        if index_block and delta_values:
            key = key[:sh] + blk[p:p + un]
            p += un
            if at_restart:  # restart point: full handle
                o, p = _varint(blk, p)
                s, p = _varint(blk, p)
            else:        # size delta only; offset follows the previous block and its trailer
                ds, p = _varint(blk, p)
                ds = ds >> 1 ^ -(ds & 1)  # zig-zag
                o = prev_off + prev_size + _TRAILER
                s = prev_size + ds
            prev_off, prev_size = o, s
            yield key, (o, s)
            continue
        vl, p = _varint(blk, p)
        key = key[:sh] + blk[p:p + un]
        p += un
        yield key, blk[p:p + vl]
        p += vl


def _handle(v: bytes):
    o, p = _varint(v, 0)
    s, _ = _varint(v, p)
    return o, s


def read_sst(path: str):
    """Yield (user_key, seq, type, value) for every entry of a block-based table file."""
    b = open(path, "rb").read()
    if len(b) < 48:
        raise DocStoreError(f"{path}: too short for an SST")
    magic = struct.unpack_from("<Q", b, len(b) - 8)[0]
    if magic == _LEGACY_MAGIC:
        f = len(b) - 48
        p = f
        mo, p = _varint(b, p)
        ms, p = _varint(b, p)
        io_, p = _varint(b, p)
        is_, p = _varint(b, p)
        index = (io_, is_)
    elif magic == _BLOCK_MAGIC:
        fv = struct.unpack_from("<I", b, len(b) - 12)[0]  # format_version
        f = len(b) - 53
        if fv >= 6:
            # checksum type | extended magic 0x3e 0x00 0x7a 0x00 | footer checksum | base context
            # checksum | metaindex size; the metaindex block sits right before the footer and the
            # index handle lives in it (key "rocksdb.index")
            if b[f + 1:f + 5] != b"\x3e\x00\x7a\x00":
                raise DocStoreError(f"{path}: bad format_version 6 footer")
            ms = struct.unpack_from("<I", b, f + 13)[0]
            mo = f - _TRAILER - ms
            index = None
        else:
            p = f + 1
            mo, p = _varint(b, p)
            ms, p = _varint(b, p)
            io_, p = _varint(b, p)
            is_, p = _varint(b, p)
            index = (io_, is_)
    else:
        raise DocStoreError(f"{path}: not a RocksDB block-based table")
    meta = dict(_block_entries(_read_block(b, mo, ms)))
    if index is None:
        if b"rocksdb.index" not in meta:
            raise DocStoreError(f"{path}: no index handle")
        index = _handle(meta[b"rocksdb.index"])
    props = {}
    if b"rocksdb.properties" in meta:
        po, ps = _handle(meta[b"rocksdb.properties"])
        props = {k: v for k, v in _block_entries(_read_block(b, po, ps))}
    delta = props.get(b"rocksdb.index.value.is.delta.encoded", b"\x00")
    delta = bool(_varint(delta, 0)[0]) if delta else False
    if props.get(b"rocksdb.block.based.table.index.type", b"\x00\x00\x00\x00")[:1] not in (b"\x00",):
        raise DocStoreError(f"{path}: only the binary-search index is supported")
    iblk = _read_block(b, *index)
    for _, h in _block_entries(iblk, index_block=True, delta_values=delta):
        if not delta:
            h = _handle(h)
        for ikey, val in _block_entries(_read_block(b, *h)):
            tr = int.from_bytes(ikey[-8:], "little")
            yield ikey[:-8], tr >> 8, tr & 0xFF, val


# --------------------------------------------------------------------------- WAL
_WAL_BLOCK = 32768


def read_wal(path: str):
    """Yield (user_key, seq, type, value) of every Put/Delete in a RocksDB write-ahead log."""
    b = open(path, "rb").read()
    p, rec = 0, bytearray()
    while p + 7 <= len(b):
        left = _WAL_BLOCK - p % _WAL_BLOCK
        if left < 7:
            p += left
            continue
        ln = struct.unpack_from("<H", b, p + 4)[0]
        t = b[p + 6]
        hdr = 7
        if t >= 5:  # recyclable record types carry a log number
            hdr, t = 11, t - 4
        if t == 0 and ln == 0:  # zero padding
            p += left
            continue
        frag = b[p + hdr:p + hdr + ln]
        p += hdr + ln
        if t == 1:
            rec = bytearray(frag)
        elif t == 2:
            rec = bytearray(frag)
            continue
        elif t == 3:
            rec += frag
            continue
        elif t == 4:
            rec += frag
        else:
            raise DocStoreError(f"{path}: bad WAL record type {t}")
        yield from _write_batch(bytes(rec))


# WriteBatch record tags (RocksDB dbformat.h ValueType)
_WB_DEL, _WB_PUT, _WB_MERGE, _WB_LOGDATA = 0x0, 0x1, 0x2, 0x3
_WB_CF_DEL, _WB_CF_PUT, _WB_CF_MERGE, _WB_SDEL, _WB_CF_SDEL = 0x4, 0x5, 0x6, 0x7, 0x8
_WB_NOOP, _WB_CF_RANGE_DEL, _WB_RANGE_DEL = 0xD, 0xE, 0xF
_WB_CF = {_WB_CF_DEL: _WB_DEL, _WB_CF_PUT: _WB_PUT, _WB_CF_SDEL: _WB_SDEL, _WB_CF_MERGE: _WB_MERGE,
          _WB_CF_RANGE_DEL: _WB_RANGE_DEL}


def _write_batch(w: bytes):
    """Yield (user_key, seq, type, value) of the default column family's Puts / Deletes of one
    WriteBatch.  Records of other column families consume their payload and sequence number but
    are not returned (rocksdict stores everything in the default family); LogData and Noop records
    carry no sequence number; merges and range deletions are refused (rocksdict issues neither)."""
    seq, count = struct.unpack_from("<QI", w, 0)
    p, i = 12, 0
    while i < count:
        if p >= len(w):
            raise DocStoreError("WriteBatch shorter than its record count")
        tag = w[p]
        p += 1
        if tag == _WB_LOGDATA:          # a blob for the log only: no key, no sequence number
            bl, p = _varint(w, p)
            p += bl
            continue
        if tag == _WB_NOOP:
            continue
        cf = 0
        if tag in _WB_CF:
            cf, p = _varint(w, p)
            tag = _WB_CF[tag]
        if tag in (_WB_MERGE, _WB_RANGE_DEL):
            raise DocStoreError(f"unsupported WriteBatch record type {tag:#x} (merge / range deletion)")
        if tag not in (_WB_PUT, _WB_DEL, _WB_SDEL):
            raise DocStoreError(f"unsupported WriteBatch record type {tag:#x}")
        kl, p = _varint(w, p)
        key = w[p:p + kl]
        p += kl
        val = b""
        if tag == _WB_PUT:
            vl, p = _varint(w, p)
            val = w[p:p + vl]
            p += vl
        if cf == 0:
            yield key, seq + i, (1 if tag == _WB_PUT else 0), val
        i += 1


# --------------------------------------------------------------------------- safe pickle
class _Global:
    def __init__(self, module, name):
        self.module, self.name = module, name

    @property
    def full(self):
        return f"{self.module}.{self.name}"


class _Reduced:
    def __init__(self, fn, args):
        self.fn, self.args, self.state = fn, args, None


_MARK = object()
_ALLOWED = {"numpy.core.multiarray._reconstruct", "numpy._core.multiarray._reconstruct", "numpy.ndarray",
            "numpy.dtype", "numpy.core.multiarray.scalar", "numpy._core.multiarray.scalar",
            "numpy.core.numeric._frombuffer", "numpy._core.numeric._frombuffer"}  # (protocol-5 arrays)


def _finish(o):
    """Turn the interpreter's symbolic objects into values (NumPy arrays)."""
    if isinstance(o, _Reduced):
        name = o.fn.full if isinstance(o.fn, _Global) else None
        if name == "numpy.dtype":
            dt = np.dtype(o.args[0])
            if o.state is not None and len(o.state) > 1 and o.state[1] in ("<", ">"):
                dt = dt.newbyteorder(o.state[1])
            return dt
        if name and name.endswith("multiarray.scalar"):  # NumPy scalar: (dtype, raw bytes)
            dt, raw = _finish(o.args[0]), o.args[1]
            if not isinstance(raw, (bytes, bytearray)):
                raise DocStoreError("numpy scalar pickle with object payload")
            return np.frombuffer(bytes(raw), dtype=dt)[0]
        if name and name.endswith("numeric._frombuffer"):  # protocol 5: (buffer, dtype, shape, order)
            if len(o.args) != 4:
                raise DocStoreError("malformed protocol-5 ndarray pickle")
            raw, dt, shape, order = o.args[0], _finish(o.args[1]), o.args[2], o.args[3]
            if not isinstance(raw, (bytes, bytearray)) or not isinstance(dt, np.dtype) or dt.hasobject:
                raise DocStoreError("protocol-5 ndarray pickle with object payload")
            a = np.frombuffer(bytes(raw), dtype=dt)
            return a.reshape(tuple(shape), order="F" if order == "F" else "C").copy()
        if name and name.endswith("multiarray._reconstruct"):
            st = o.state
            if st is None or len(st) < 5:
                raise DocStoreError("ndarray pickle without state")
            shape, dt, fortran, raw = st[1], _finish(st[2]), st[3], st[4]
            if not isinstance(raw, (bytes, bytearray)):
                raise DocStoreError("ndarray pickle with object payload")
            a = np.frombuffer(bytes(raw), dtype=dt)
            return a.reshape(shape, order="F" if fortran else "C").copy()
        raise DocStoreError(f"pickle global {name} is not allowed")
    if isinstance(o, dict):
        return {_finish(k): _finish(v) for k, v in o.items()}
    if isinstance(o, list):
        return [_finish(v) for v in o]
    if isinstance(o, tuple):
        return tuple(_finish(v) for v in o)
    if isinstance(o, _Global):
        raise DocStoreError(f"bare pickle global {o.full}")
    return o


def safe_unpickle(blob: bytes):
    """Decode a pickle of plain containers / scalars / NumPy arrays without executing anything."""
    stack, memo = [], {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _ in pickletools.genops(io.BytesIO(blob)):
        nm = op.name
        if nm in ("PROTO", "FRAME"):
            continue
        if nm == "STOP":
            return _finish(stack.pop())
        if nm == "MARK":
            stack.append(_MARK)
        elif nm in ("EMPTY_DICT",):
            stack.append({})
        elif nm == "EMPTY_LIST":
            stack.append([])
        elif nm == "EMPTY_TUPLE":
            stack.append(())
        elif nm in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING", "BINSTRING"):
            stack.append(arg)
        elif nm in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8", "BYTEARRAY8"):
            stack.append(bytes(arg))
        elif nm in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG", "BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif nm == "NONE":
            stack.append(None)
        elif nm == "NEWTRUE":
            stack.append(True)
        elif nm == "NEWFALSE":
            stack.append(False)
        elif nm == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif nm in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[arg] = stack[-1]
        elif nm in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[arg])
        elif nm == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif nm in ("TUPLE1", "TUPLE2", "TUPLE3"):
            n = int(nm[-1])
            t = tuple(stack[-n:])
            del stack[-n:]
            stack.append(t)
        elif nm == "LIST":
            stack.append(list(pop_mark()))
        elif nm == "DICT":
            it = pop_mark()
            stack.append({it[i]: it[i + 1] for i in range(0, len(it), 2)})
        elif nm == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif nm == "APPENDS":
            it = pop_mark()
            stack[-1].extend(it)
        elif nm == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif nm == "SETITEMS":
            it = pop_mark()
            for i in range(0, len(it), 2):
                stack[-1][it[i]] = it[i + 1]
        elif nm == "GLOBAL":
            mod, name = arg.split(" ", 1) if " " in arg else arg.split("\n", 1)
            g = _Global(mod, name)
            if g.full not in _ALLOWED:
                raise DocStoreError(f"pickle global {g.full} is not allowed")
            stack.append(g)
        elif nm == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            g = _Global(mod, name)
            if g.full not in _ALLOWED:
                raise DocStoreError(f"pickle global {g.full} is not allowed")
            stack.append(g)
        elif nm == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(_Reduced(fn, args))
        elif nm == "BUILD":
            st = stack.pop()
            if not isinstance(stack[-1], _Reduced):
                raise DocStoreError("BUILD on a non-reduced object")
            stack[-1].state = st
        else:
            raise DocStoreError(f"pickle opcode {nm} is not supported")
    raise DocStoreError("pickle without STOP")


# --------------------------------------------------------------------------- rocksdict encoding
def decode_rocksdict(b: bytes):
    """rocksdict's (non-raw mode) encoding of a key or value: a type byte, then the payload."""
    if not b:
        raise DocStoreError("empty rocksdict value")
    t, p = b[0], b[1:]
    if t == 0x01:
        return bytes(p)
    if t == 0x02:
        return p.decode("utf-8")
    if t in (0x03, 0x04):
        # rocksdict's int / float payloads: their byte order is pinned by no reference artefact (the
        # reference's folders use str keys and pickled values), so they are refused, not guessed
        raise DocStoreError(f"rocksdict {'int' if t == 0x03 else 'float'} encoding is not supported (byte order unpinned)")
    if t == 0x05:
        return bool(p[0])
    if t == 0x06:
        return safe_unpickle(p)
    raise DocStoreError(f"unknown rocksdict type byte {t:#x}")


class RocksDictReader:
    """The live entries of a rocksdict directory, read once: ``{key: value}`` (decoded).

    Every ``*.sst`` and ``*.log`` in the directory is read and each key resolves to its highest
    sequence number.  Limitation: the live file set in MANIFEST is not consulted, so a table or log
    that a crash left behind (or a flushed WAL still on disk) is read as well; that is exact for the
    reference's persisted folders (one table, no stale files) but could revive a key whose tombstone a
    bottommost compaction dropped.  A directory with several logs is reported with a warning."""

    def __init__(self, path: str):
        if not os.path.isdir(path):
            raise DocStoreError(f"{path} is not a directory")
        best = {}
        srcs = [read_sst(f) for f in sorted(glob.glob(os.path.join(path, "*.sst")))]
        logs = sorted(glob.glob(os.path.join(path, "*.log")))
        if len(logs) > 1:
            logger.warning("%s holds %d write-ahead logs; the reader does not consult MANIFEST's live set", path,
                           len(logs))
        srcs += [read_wal(f) for f in logs]
        for it in srcs:
            for key, seq, typ, val in it:
                if typ not in (0, 1, 7):
                    continue
                if key not in best or seq > best[key][0]:
                    best[key] = (seq, typ, val)
        self.data = {}
        for key, (seq, typ, val) in best.items():
            if typ == 1:
                self.data[decode_rocksdict(key)] = val

    def __len__(self):
        return len(self.data)

    def __contains__(self, k):
        return k in self.data

    def keys(self):
        return self.data.keys()

    def get(self, k, default=None):
        v = self.data.get(k)
        return default if v is None else decode_rocksdict(v)

    def __getitem__(self, k):
        return decode_rocksdict(self.data[k])

    def items(self):
        for k, v in self.data.items():
            yield k, decode_rocksdict(v)


def is_rocksdict_dir(path: str) -> bool:
    return os.path.isdir(path) and (os.path.exists(os.path.join(path, "CURRENT")) or
                                    bool(glob.glob(os.path.join(path, "*.sst"))))
