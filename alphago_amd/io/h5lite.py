"""Self-contained HDF5 subset (reader + writer), no libhdf5 / h5py needed.

Why: the reference stores training data and Keras weights in HDF5 via h5py
(game_converter.py:66-88, policy.py:167,189).  h5py is not
installed in this environment, so this module implements exactly the part of
the format those files use:

Reader
  * superblock v0/v1, 8-byte offsets/lengths
  * v1 object headers (+ continuation blocks)
  * old-style groups: symbol-table message -> v1 B-tree (type 0, any depth)
    -> symbol-table nodes -> local-heap names
  * datasets with compact / contiguous / chunked (v1 B-tree type 1) layout,
    filters LZF (32000, native decoder), deflate (1), shuffle (2)
  * datatypes: fixed-point, IEEE float, fixed-length strings; attributes v1-v3
  * chunk-sliced row reads (``H5Dataset.rows`` / ``read_rows``): only the
    chunks that hold the requested rows are read and decoded, on a native
    thread pool (``lzf_decompress_many``) — never the whole dataset
Writer (h5py/Keras-1.0 readable)
  * superblock v0, v1 object headers, symbol-table groups with multi-level
    B-trees (sorted names), contiguous datasets, attributes
  * streamed datasets: rows appended straight to the file (the converter
    writes millions of positions without holding them in memory), either
    contiguous or chunked along rows with the LZF filter — the reference's
    layout, ``chunks=(64, F, S, S)`` / ``(1024, 2)``, ``compression="lzf"``,
    ``maxshape=(None, ...)`` (game_converter.py:71-86)
"""
from __future__ import annotations

import io
import os
import struct
import zlib
from typing import Dict, Iterable, List, Optional, Tuple, Union

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
SIG = b"\x89HDF\r\n\x1a\n"


# ===================================================================== reader
class H5Error(Exception):
    pass


def _lzf(data: bytes, out_len: int) -> bytes:
    from .._native import engine

    return engine().lzf_decompress(data, out_len)


class _Type:
    def __init__(self, cls: int, size: int, dtype, is_str: bool = False):
        self.cls, self.size, self.dtype, self.is_str = cls, size, dtype, is_str


def _parse_datatype(b: bytes, off: int = 0) -> _Type:
    cv = b[off]
    cls, ver = cv & 0x0F, cv >> 4
    bits = b[off + 1] | (b[off + 2] << 8) | (b[off + 3] << 16)
    size = struct.unpack_from("<I", b, off + 4)[0]
    endian = ">" if bits & 1 else "<"
    if cls == 0:  # fixed point
        signed = bool(bits & 0x08)
        return _Type(cls, size, np.dtype("%s%s%d" % (endian, "i" if signed else "u", size)))
    if cls == 1:  # float
        return _Type(cls, size, np.dtype("%sf%d" % (endian, size)))
    if cls == 3:  # fixed-length string
        return _Type(cls, size, np.dtype("S%d" % size), True)
    if cls == 4:  # bitfield
        return _Type(cls, size, np.dtype("%su%d" % (endian, size)))
    if cls == 8:  # enum (h5py bool) — base type follows the header
        base = _parse_datatype(b, off + 8)
        return _Type(cls, size, base.dtype)
    raise H5Error("unsupported datatype class %d" % cls)


def _parse_dataspace(b: bytes, off: int = 0) -> Tuple[int, ...]:
    ver = b[off]
    rank = b[off + 1]
    flags = b[off + 2]
    if ver == 1:
        p = off + 8
    elif ver == 2:
        if b[off + 3] == 0:  # scalar
            return ()
        if b[off + 3] == 2:  # null
            return (0,)
        p = off + 4
    else:
        raise H5Error("dataspace version %d" % ver)
    return tuple(struct.unpack_from("<%dQ" % rank, b, p)) if rank else ()


class H5Object:
    """A group or dataset in an opened file."""

    def __init__(self, f: "H5File", addr: int, name: str):
        self.file, self.addr, self.name = f, addr, name
        self.msgs = f._read_object_header(addr)
        self._attrs = None

    # -------- common
    @property
    def attrs(self) -> Dict[str, object]:
        if self._attrs is None:
            self._attrs = {}
            for mtype, data in self.msgs:
                if mtype == 0x000C:
                    k, v = self.file._parse_attribute(data)
                    self._attrs[k] = v
        return self._attrs

    def _msg(self, t):
        for mtype, data in self.msgs:
            if mtype == t:
                return data
        return None


class H5Group(H5Object):
    def __init__(self, f, addr, name):
        super().__init__(f, addr, name)
        st = self._msg(0x0011)
        if st is None:
            raise H5Error("%s is not an old-style group (no symbol table message)" % name)
        self.btree, self.heap = struct.unpack_from("<QQ", st, 0)
        self._links = None

    def _entries(self) -> Dict[str, int]:
        if self._links is None:
            heap = self.file._read_local_heap(self.heap)
            out: Dict[str, int] = {}
            self.file._walk_group_btree(self.btree, heap, out)
            self._links = out
        return self._links

    def keys(self) -> List[str]:
        return list(self._entries().keys())

    def __contains__(self, k) -> bool:
        return k in self._entries()

    def __iter__(self):
        return iter(self.keys())

    def __len__(self):
        return len(self._entries())

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def __getitem__(self, path: str):
        node = self
        for part in [p for p in path.split("/") if p]:
            if not isinstance(node, H5Group):
                raise KeyError(path)
            ents = node._entries()
            if part not in ents:
                raise KeyError(path)
            node = self.file._open(ents[part], part)
        return node


class H5Dataset(H5Object):
    def __init__(self, f, addr, name):
        super().__init__(f, addr, name)
        self.shape = _parse_dataspace(self._msg(0x0001))
        self._type = _parse_datatype(self._msg(0x0003))
        self.dtype = self._type.dtype
        self._layout = self._parse_layout(self._msg(0x0008))
        self._filters = self._parse_filters(self._msg(0x000B))
        self._cache = None
        self._chunk_index = None
        self._chunk_of_row = None

    def __len__(self):
        return self.shape[0] if self.shape else 1

    @property
    def ndim(self):
        return len(self.shape)

    def _parse_layout(self, b: bytes):
        ver = b[0]
        if ver in (1, 2):
            rank, cls = b[1], b[2]
            p = 8
            addr = None
            if cls != 0:
                addr = struct.unpack_from("<Q", b, p)[0]
                p += 8
            dims = struct.unpack_from("<%dI" % rank, b, p)
            p += 4 * rank
            if cls == 0:
                size = struct.unpack_from("<I", b, p)[0]
                return ("compact", b[p + 4:p + 4 + size])
            if cls == 1:
                return ("contiguous", addr, int(np.prod(self.shape)) * self._type.size)
            return ("chunked", addr, dims)
        if ver == 3:
            cls = b[1]
            if cls == 0:
                size = struct.unpack_from("<H", b, 2)[0]
                return ("compact", b[4:4 + size])
            if cls == 1:
                addr, size = struct.unpack_from("<QQ", b, 2)
                return ("contiguous", addr, size)
            if cls == 2:
                rank = b[2]
                addr = struct.unpack_from("<Q", b, 3)[0]
                dims = struct.unpack_from("<%dI" % rank, b, 11)
                return ("chunked", addr, dims)
        raise H5Error("unsupported layout version %d" % ver)

    def _parse_filters(self, b: Optional[bytes]):
        if b is None:
            return []
        ver, n = b[0], b[1]
        out = []
        p = 8 if ver == 1 else 2
        for _ in range(n):
            fid = struct.unpack_from("<H", b, p)[0]
            if ver == 1 or fid >= 256:
                namelen = struct.unpack_from("<H", b, p + 2)[0]
                p += 4
            else:
                namelen = 0
                p += 2
            flags, nvals = struct.unpack_from("<HH", b, p)
            p += 4
            if namelen:
                p += ((namelen + 7) // 8 * 8) if ver == 1 else namelen
            vals = struct.unpack_from("<%dI" % nvals, b, p)
            p += 4 * nvals
            if ver == 1 and nvals % 2:
                p += 4
            out.append((fid, vals))
        return out

    def _unfilter(self, raw: bytes, mask: int, nbytes: int) -> bytes:
        for i in reversed(range(len(self._filters))):
            if mask & (1 << i):
                continue
            fid, vals = self._filters[i]
            if fid == 32000:
                raw = _lzf(raw, nbytes)
            elif fid == 1:
                raw = zlib.decompress(raw)
            elif fid == 2:
                es = vals[0] if vals else self._type.size
                a = np.frombuffer(raw, np.uint8)
                n = len(a) // es
                raw = a[: n * es].reshape(es, n).T.tobytes() + a[n * es:].tobytes()
            else:
                raise H5Error("unsupported filter %d" % fid)
        return raw

    def read(self) -> np.ndarray:
        if self._cache is not None:
            return self._cache
        lay = self._layout
        n = int(np.prod(self.shape)) if self.shape else 1
        if lay[0] == "compact":
            arr = np.frombuffer(lay[1], self.dtype, count=n)
        elif lay[0] == "contiguous":
            if lay[1] == UNDEF:
                arr = np.zeros(n, self.dtype)
            else:
                arr = self.file._mm(lay[1], n * self._type.size, self.dtype)
        else:
            arr = self._read_chunked(lay[1], lay[2])
        arr = arr.reshape(self.shape) if self.shape else arr.reshape(())
        self._cache = arr
        return arr

    def _read_chunked(self, btree: int, cdims) -> np.ndarray:
        rank = len(self.shape)
        chunk = tuple(cdims[:rank])
        out = np.zeros(self.shape, self.dtype)
        cbytes = int(np.prod(chunk)) * self._type.size
        for offs, addr, size, mask in self.file._walk_chunk_btree(btree, rank):
            raw = self.file._read(addr, size)
            if self._filters:
                raw = self._unfilter(raw, mask, cbytes)
            a = np.frombuffer(raw, self.dtype, count=int(np.prod(chunk))).reshape(chunk)
            sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, chunk, self.shape))
            out[sl] = a[tuple(slice(0, s.stop - s.start) for s in sl)]
        return out

    # ---------------------------------------------------- chunk-sliced reads
    @property
    def chunked(self) -> bool:
        return self._layout[0] == "chunked"

    @property
    def chunk_rows(self) -> int:
        """Rows per chunk (chunked datasets must be chunked along dim 0 only)."""
        if not self.chunked:
            return len(self)
        cd = tuple(self._layout[2][:len(self.shape)])
        if cd[1:] != tuple(self.shape[1:]):
            raise H5Error("row reads need chunks spanning whole rows (chunk %s, shape %s)" % (cd, self.shape))
        return int(cd[0])

    def chunk_index(self):
        """(row offset, file address, stored size, filter mask) per chunk, by row offset."""
        if self._chunk_index is None:
            ents = sorted(((int(o[0]), a, sz, m) for o, a, sz, m in
                           self.file._walk_chunk_btree(self._layout[1], len(self.shape))), key=lambda e: e[0])
            self._chunk_index = ents
            self._chunk_of_row = {e[0] // self.chunk_rows: i for i, e in enumerate(ents)}
        return self._chunk_index

    def read_chunks(self, chunk_ids, threads: int = 8, out: Optional[np.ndarray] = None,
                    slots=None) -> np.ndarray:
        """Decode the given chunks (by chunk number = row offset // chunk_rows).
        Chunk i lands at rows [s*chunk_rows, (s+1)*chunk_rows) of ``out``, with
        s = slots[i] (default i); ``out`` defaults to a new array of
        ``len(chunk_ids) * chunk_rows`` rows.  A chunk never written reads as
        zeros.  Pass a long-lived ``out``: the first-touch page faults of a fresh
        allocation serialise the decode threads."""
        idx = self.chunk_index()
        cr = self.chunk_rows
        row_shape = tuple(self.shape[1:])
        row_elems = int(np.prod(row_shape)) if row_shape else 1
        cbytes = cr * row_elems * self._type.size
        if out is None:
            out = np.empty((len(chunk_ids) * cr,) + row_shape, self.dtype)
        slots = list(range(len(chunk_ids))) if slots is None else [int(x) for x in slots]
        lzf_only = len(self._filters) == 1 and self._filters[0][0] == 32000
        raws, raw_slots = [], []
        for k, c in enumerate(chunk_ids):
            sl = slots[k]
            e = self._chunk_of_row.get(int(c))
            if e is None:
                out[sl * cr:(sl + 1) * cr] = 0
                continue
            off, addr, size, mask = idx[e]
            raw = self.file._read(addr, size)
            if lzf_only and not (mask & 1):
                raws.append(raw)
                raw_slots.append(sl)
            else:
                raw = self._unfilter(raw, mask, cbytes) if self._filters else raw
                out[sl * cr:(sl + 1) * cr] = np.frombuffer(raw, self.dtype, count=cr * row_elems).reshape(
                    (cr,) + row_shape)
        if raws:
            from .._native import engine

            engine().lzf_decompress_into(raws, out.reshape(-1).view(np.uint8), cbytes, threads, raw_slots)
        return out

    def read_rows(self, start: int, stop: int, threads: int = 8) -> np.ndarray:
        """Rows [start, stop) decoding only the chunks that hold them."""
        stop = min(stop, len(self))
        if stop <= start:
            return np.zeros((0,) + tuple(self.shape[1:]), self.dtype)
        if not self.chunked:
            return self.read()[start:stop]
        cr = self.chunk_rows
        c0, c1 = start // cr, (stop - 1) // cr + 1
        block = self.read_chunks(list(range(c0, c1)), threads)
        return block[start - c0 * cr:stop - c0 * cr]

    def rows(self, idx, threads: int = 8) -> np.ndarray:
        """Arbitrary rows (any order, repeats allowed), decoding each needed
        chunk once."""
        idx = np.asarray(idx, np.int64)
        if not self.chunked:
            return self.read()[idx]
        cr = self.chunk_rows
        cids, inv = np.unique(idx // cr, return_inverse=True)
        block = self.read_chunks(cids.tolist(), threads)
        return block[inv * cr + idx % cr]

    def __getitem__(self, idx):
        return self.read()[idx]

    def __array__(self, dtype=None):
        a = self.read()
        return a.astype(dtype) if dtype is not None else a


class H5File(H5Group):
    """Read-only HDF5 file (subset).  API mirrors h5py for the bits we use."""

    def __init__(self, path: str, mode: str = "r"):
        if mode != "r":
            raise ValueError("H5File is read-only; use H5Writer")
        self.path = path
        self._fh = open(path, "rb")
        self._data = np.memmap(path, dtype=np.uint8, mode="r") if os.path.getsize(path) else b""
        sb = self._read(0, 96)
        if sb[:8] != SIG:
            raise H5Error("not an HDF5 file: %s" % path)
        ver = sb[8]
        if ver not in (0, 1):
            raise H5Error("superblock version %d not supported" % ver)
        if sb[13] != 8 or sb[14] != 8:
            raise H5Error("only 8-byte offsets/lengths supported")
        p = 24 if ver == 0 else 28
        root_entry = p + 32
        root_obj = struct.unpack_from("<Q", sb, root_entry + 8)[0]
        H5Group.__init__(self, self, root_obj, "/")

    def close(self):
        self._fh.close()
        self._data = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -------- low level
    def _read(self, addr: int, n: int) -> bytes:
        return bytes(self._data[addr:addr + n])

    def _mm(self, addr: int, nbytes: int, dtype) -> np.ndarray:
        return np.frombuffer(self._data[addr:addr + nbytes], dtype)  # zero-copy view of the mmap

    def _open(self, addr: int, name: str):
        msgs = self._read_object_header(addr)
        if any(t == 0x0011 for t, _ in msgs):
            return H5Group(self, addr, name)
        return H5Dataset(self, addr, name)

    def _read_object_header(self, addr: int):
        hdr = self._read(addr, 16)
        ver = hdr[0]
        if ver != 1:
            raise H5Error("object header version %d not supported" % ver)
        nmsgs, _, hsize = struct.unpack_from("<HII", hdr, 2)
        blocks = [(addr + 16, hsize)]
        msgs = []
        while blocks and len(msgs) < nmsgs:
            start, size = blocks.pop(0)
            b = self._read(start, size)
            p = 0
            while p + 8 <= size and len(msgs) < nmsgs:
                mtype, msize, flags = struct.unpack_from("<HHB", b, p)
                data = b[p + 8:p + 8 + msize]
                if mtype == 0x0010:
                    caddr, clen = struct.unpack_from("<QQ", data, 0)
                    blocks.append((caddr, clen))
                msgs.append((mtype, data))
                p += 8 + msize
        return msgs

    def _read_local_heap(self, addr: int) -> bytes:
        h = self._read(addr, 32)
        if h[:4] != b"HEAP":
            raise H5Error("bad local heap")
        size, _, daddr = struct.unpack_from("<QQQ", h, 8)
        return self._read(daddr, size)

    @staticmethod
    def _heap_str(heap: bytes, off: int) -> str:
        end = heap.index(b"\0", off)
        return heap[off:end].decode("utf-8", "replace")

    def _walk_group_btree(self, addr: int, heap: bytes, out: Dict[str, int]) -> None:
        h = self._read(addr, 24)
        if h[:4] != b"TREE":
            raise H5Error("bad group B-tree node")
        ntype, level, used = h[4], h[5], struct.unpack_from("<H", h, 6)[0]
        body = self._read(addr + 24, used * 16 + 8)
        for i in range(used):
            child = struct.unpack_from("<Q", body, 8 + 16 * i)[0]
            if level > 0:
                self._walk_group_btree(child, heap, out)
            else:
                sn = self._read(child, 8)
                if sn[:4] != b"SNOD":
                    raise H5Error("bad symbol node")
                nsym = struct.unpack_from("<H", sn, 6)[0]
                ents = self._read(child + 8, 40 * nsym)
                for k in range(nsym):
                    noff, oaddr = struct.unpack_from("<QQ", ents, 40 * k)
                    out[self._heap_str(heap, noff)] = oaddr

    def _walk_chunk_btree(self, addr: int, rank: int):
        if addr == UNDEF:  # no chunk written yet (libhdf5: UNDEF index address in the layout)
            return
        h = self._read(addr, 24)
        if h[:4] != b"TREE":
            raise H5Error("bad chunk B-tree node")
        level, used = h[5], struct.unpack_from("<H", h, 6)[0]
        ksize = 8 + 8 * (rank + 1)
        body = self._read(addr + 24, used * (ksize + 8) + ksize)
        for i in range(used):
            kp = i * (ksize + 8)
            csize, mask = struct.unpack_from("<II", body, kp)
            offs = struct.unpack_from("<%dQ" % rank, body, kp + 8)
            child = struct.unpack_from("<Q", body, kp + ksize)[0]
            if level > 0:
                yield from self._walk_chunk_btree(child, rank)
            else:
                yield offs, child, csize, mask

    def _parse_attribute(self, b: bytes):
        ver = b[0]
        nlen, tlen, slen = struct.unpack_from("<HHH", b, 2)
        p = 8
        if ver == 3:
            p = 9
        pad = (lambda x: (x + 7) // 8 * 8) if ver == 1 else (lambda x: x)
        name = b[p:p + nlen].split(b"\0")[0].decode("utf-8", "replace")
        p += pad(nlen)
        t = _parse_datatype(b, p)
        p += pad(tlen)
        shape = _parse_dataspace(b, p)
        p += pad(slen)
        n = int(np.prod(shape)) if shape else 1
        arr = np.frombuffer(b[p:p + n * t.size], t.dtype, count=n)
        if not shape:
            v = arr[0]
            return name, (v.decode() if t.is_str else v.item())
        return name, arr.reshape(shape).copy()


def open_file(path: str) -> H5File:
    return H5File(path)


# ===================================================================== writer
def _pad8(n: int) -> int:
    return (n + 7) // 8 * 8


def _dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.kind in "iu":
        bits = 0x08 if dt.kind == "i" else 0
        if dt.byteorder == ">":
            bits |= 1
        return bytes([0x10, bits, 0, 0]) + struct.pack("<IHH", dt.itemsize, 0, dt.itemsize * 8)
    if dt.kind == "b":
        return bytes([0x10, 0, 0, 0]) + struct.pack("<IHH", 1, 0, 8)
    if dt.kind == "f":
        if dt.itemsize == 4:
            return bytes([0x11, 0x20, 0x1F, 0x00]) + struct.pack("<IHHBBBBI", 4, 0, 32, 23, 8, 0, 23, 127)
        if dt.itemsize == 8:
            return bytes([0x11, 0x20, 0x3F, 0x00]) + struct.pack("<IHHBBBBI", 8, 0, 64, 52, 11, 0, 52, 1023)
        if dt.itemsize == 2:
            return bytes([0x11, 0x20, 0x0F, 0x00]) + struct.pack("<IHHBBBBI", 2, 0, 16, 10, 5, 0, 10, 15)
    if dt.kind == "S":
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", dt.itemsize)  # null-padded ascii
    raise H5Error("cannot write dtype %s" % dt)


def _space_msg(shape, maxshape=None) -> bytes:
    shape = tuple(int(s) for s in shape)
    b = bytes([1, len(shape), 1 if maxshape is not None else 0, 0]) + b"\0" * 4
    b += b"".join(struct.pack("<Q", s) for s in shape)
    if maxshape is not None:
        b += b"".join(struct.pack("<Q", UNDEF if m is None else int(m)) for m in maxshape)
    return b


LZF_ID = 32000


def _lzf_filter_msg(chunk_bytes: int) -> bytes:
    """Filter-pipeline message v1 with the h5py LZF filter (optional flag set,
    client values: filter version 4, LZF 0x0105, chunk bytes)."""
    name = b"lzf\0" + b"\0" * 4
    vals = (4, 0x0105, chunk_bytes)
    b = struct.pack("<BB6x", 1, 1)
    b += struct.pack("<HHHH", LZF_ID, len(name), 1, len(vals)) + name
    b += struct.pack("<%dI" % len(vals), *vals) + b"\0" * (4 if len(vals) % 2 else 0)
    return b


def _as_attr_array(v) -> np.ndarray:
    if isinstance(v, str):
        return np.array(v.encode("utf-8"))
    if isinstance(v, bytes):
        return np.array(v)
    a = np.asarray(v)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "utf-8")
    if a.dtype.kind == "O":
        a = np.array([x.encode() if isinstance(x, str) else x for x in a.ravel()]).reshape(a.shape)
    return a


class _WDataset:
    def __init__(self, name, shape, dtype, data=None, addr=None):
        self.name, self.shape, self.dtype = name, tuple(shape), np.dtype(dtype)
        self.data, self.addr = data, addr
        self.attrs: Dict[str, object] = {}
        self.chunk_rows = 0          # >0: chunked along dim 0
        self.compression = None      # None or "lzf"
        self.chunks: List[Tuple[int, int, int, int]] = []  # (row offset, addr, stored size, filter mask)


class _WGroup:
    def __init__(self, writer: "H5Writer", name: str):
        self.w, self.name = writer, name
        self.children: Dict[str, Union["_WGroup", _WDataset]] = {}
        self.attrs: Dict[str, object] = {}

    def create_group(self, name: str) -> "_WGroup":
        parts = [p for p in name.split("/") if p]
        g = self
        for p in parts:
            if p not in g.children:
                g.children[p] = _WGroup(self.w, p)
            g = g.children[p]
        return g

    require_group = create_group

    def create_dataset(self, name: str, data=None, shape=None, dtype=None) -> _WDataset:
        parts = [p for p in name.split("/") if p]
        g = self.create_group("/".join(parts[:-1])) if len(parts) > 1 else self
        if data is not None:
            arr = np.ascontiguousarray(np.asarray(data, dtype=dtype) if dtype is not None else np.asarray(data))
            d = _WDataset(parts[-1], arr.shape, arr.dtype, data=arr)
        else:
            d = _WDataset(parts[-1], shape, dtype)
        g.children[parts[-1]] = d
        return d

    def __setitem__(self, name, value):
        self.create_dataset(name, data=value)

    def __contains__(self, name):
        return name in self.children

    def __getitem__(self, name):
        return self.children[name]


class StreamedDataset:
    """Rows appended directly to the file; finalised by H5Writer.close().

    Contiguous (default) or chunked along rows (``chunk_rows``) with optional
    LZF compression: each full chunk is compressed and written as soon as it
    is complete (a chunk that does not shrink is stored raw with its filter
    mask bit set, as libhdf5 does for an optional filter); the partial last
    chunk is zero-padded to the full chunk shape, as HDF5 requires."""

    def __init__(self, writer: "H5Writer", ds: _WDataset, row_shape, dtype, chunk_rows: int = 0,
                 compression: Optional[str] = None):
        self.w, self.ds = writer, ds
        self.row_shape, self.dtype = tuple(row_shape), np.dtype(dtype)
        self.rows = 0
        if compression not in (None, "lzf"):
            raise H5Error("unsupported compression %r" % compression)
        if compression and not chunk_rows:
            raise H5Error("compression needs a chunked layout")
        ds.chunk_rows, ds.compression = int(chunk_rows), compression
        self._pending: List[np.ndarray] = []
        self._npending = 0
        self.ds.addr = writer._tell()
        writer._stream_open = self

    def append(self, rows: np.ndarray) -> None:
        rows = np.ascontiguousarray(rows, dtype=self.dtype)
        if rows.shape[1:] != self.row_shape:
            raise ValueError("row shape mismatch %s vs %s" % (rows.shape[1:], self.row_shape))
        if self.w._stream_open is not self:
            raise H5Error("only the most recently created streamed dataset can be appended to")
        if not self.ds.chunk_rows:
            self.w._fh.write(rows.tobytes())
            self.rows += rows.shape[0]
            return
        self._pending.append(rows)
        self._npending += rows.shape[0]
        cr = self.ds.chunk_rows
        if self._npending >= cr:
            buf = np.concatenate(self._pending)
            nfull = (len(buf) // cr) * cr
            for o in range(0, nfull, cr):
                self._write_chunk(buf[o:o + cr], cr)
            rest = buf[nfull:]
            self._pending = [rest] if len(rest) else []
            self._npending = len(rest)

    def _write_chunk(self, block: np.ndarray, nrows: int) -> None:
        cr = self.ds.chunk_rows
        if len(block) < cr:
            block = np.concatenate([block, np.zeros((cr - len(block),) + self.row_shape, self.dtype)])
        raw = np.ascontiguousarray(block).tobytes()
        mask = 0
        if self.ds.compression == "lzf":
            from .._native import engine

            c = engine().lzf_compress(raw)
            if c:
                raw = c
            else:
                mask = 1  # filter 0 skipped for this chunk
        addr = self.w._alloc(raw)
        self.ds.chunks.append((self.rows, addr, len(raw), mask))
        self.rows += nrows

    def __len__(self):
        return self.rows + (self._npending if self.ds.chunk_rows else 0)

    def finish(self):
        if self.ds.chunk_rows and self._npending:
            n = self._npending
            buf = np.concatenate(self._pending)
            self._pending, self._npending = [], 0
            self._write_chunk(buf, n)
        self.ds.shape = (self.rows,) + self.row_shape
        if self.rows == 0 and not self.ds.chunk_rows:
            self.ds.addr = UNDEF
        if self.w._stream_open is self:
            self.w._stream_open = None


class H5Writer(_WGroup):
    """Write-once HDF5 file (h5py-compatible subset).  Usage::

        with H5Writer(path) as f:
            f.attrs["layer_names"] = [b"a", b"b"]
            g = f.create_group("a"); g["a_W"] = np.zeros((3, 3), np.float32)
            s = f.stream_dataset("states", (48, 19, 19), np.uint8); s.append(batch)
    """

    LEAF_K = 32      # symbol-table node capacity = 2K entries
    INTERNAL_K = 32  # B-tree node capacity = 2K children

    def __init__(self, path: str):
        _WGroup.__init__(self, self, "/")
        self.path = path
        self._fh = open(path, "wb")
        self._fh.write(b"\0" * 96)  # superblock placeholder
        self._stream_open = None
        self._closed = False

    def _tell(self) -> int:
        return self._fh.tell()

    def stream_dataset(self, name: str, row_shape, dtype, chunk_rows: int = 0,
                       compression: Optional[str] = None) -> StreamedDataset:
        if self._stream_open is not None:
            self._stream_open.finish()
        d = self.create_dataset(name, shape=(0,) + tuple(row_shape), dtype=dtype)
        return StreamedDataset(self, d, row_shape, dtype, chunk_rows, compression)

    def create_chunked(self, name: str, data, chunk_rows: int, compression: Optional[str] = "lzf") -> _WDataset:
        """Whole-array convenience: a chunked (+LZF) dataset from ``data``."""
        data = np.ascontiguousarray(data)
        s = self.stream_dataset(name, data.shape[1:], data.dtype, chunk_rows, compression)
        s.append(data)
        s.finish()
        return s.ds

    # ---- layout helpers
    def _alloc(self, data: bytes) -> int:
        addr = self._fh.tell()
        self._fh.write(data)
        pad = _pad8(len(data)) - len(data)
        if pad:
            self._fh.write(b"\0" * pad)
        return addr

    def _attr_msg(self, name: str, value) -> bytes:
        arr = _as_attr_array(value)
        nb = name.encode("utf-8") + b"\0"
        tb = _dtype_msg(arr.dtype)
        sb = _space_msg(arr.shape) if arr.shape else bytes([1, 0, 0, 0, 0, 0, 0, 0])
        body = struct.pack("<BBHHH", 1, 0, len(nb), len(tb), len(sb))
        body += nb + b"\0" * (_pad8(len(nb)) - len(nb))
        body += tb + b"\0" * (_pad8(len(tb)) - len(tb))
        body += sb + b"\0" * (_pad8(len(sb)) - len(sb))
        body += arr.tobytes()
        return body

    def _object_header(self, msgs: List[Tuple[int, bytes]]) -> int:
        body = b""
        for t, data in msgs:
            pd = _pad8(len(data))
            body += struct.pack("<HHB3x", t, pd, 0) + data + b"\0" * (pd - len(data))
        hdr = struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4
        return self._alloc(hdr + body)

    def _write_chunk_btree(self, d: _WDataset) -> int:
        """v1 B-tree (type 1) over the dataset's chunks; full-capacity nodes
        (2K entries, K = 32) so libhdf5 can read them."""
        rank = len(d.shape) + 1
        ksize = 8 + 8 * rank
        cap = 64
        node_size = 24 + cap * 8 + (cap + 1) * ksize
        cr = d.chunk_rows

        def key(row_off, size=0, mask=0):
            return struct.pack("<II", size, mask) + struct.pack("<%dQ" % rank, row_off, *([0] * (rank - 1)))

        if not d.chunks:  # empty dataset: libhdf5 writes an UNDEF index address, not a fake chunk record
            return UNDEF
        # level 0: (first key, last-bound key, node addr)
        ents = d.chunks
        level, nodes = 0, []
        groups = [ents[i:i + cap] for i in range(0, len(ents), cap)]
        base = self._tell()
        addrs = [base + k * _pad8(node_size) for k in range(len(groups))]
        for k, grp in enumerate(groups):
            left = addrs[k - 1] if k > 0 else UNDEF
            right = addrs[k + 1] if k + 1 < len(groups) else UNDEF
            b = b"TREE" + struct.pack("<BBHQQ", 1, 0, len(grp), left, right)
            for off, addr, size, mask in grp:
                b += key(off, size, mask) + struct.pack("<Q", addr)
            end = grp[-1][0] + cr
            b += key(end)
            b += b"\0" * (node_size - len(b))
            a = self._alloc(b)
            assert a == addrs[k]
            nodes.append((grp[0][0], end, a))
        while len(nodes) > 1:
            level += 1
            groups = [nodes[i:i + cap] for i in range(0, len(nodes), cap)]
            base = self._tell()
            addrs = [base + k * _pad8(node_size) for k in range(len(groups))]
            nxt = []
            for k, grp in enumerate(groups):
                left = addrs[k - 1] if k > 0 else UNDEF
                right = addrs[k + 1] if k + 1 < len(groups) else UNDEF
                b = b"TREE" + struct.pack("<BBHQQ", 1, level, len(grp), left, right)
                for first, _, addr in grp:
                    b += key(first) + struct.pack("<Q", addr)
                b += key(grp[-1][1])
                b += b"\0" * (node_size - len(b))
                a = self._alloc(b)
                assert a == addrs[k]
                nxt.append((grp[0][0], grp[-1][1], a))
            nodes = nxt
        return nodes[0][2]

    def _write_dataset(self, d: _WDataset) -> int:
        if d.chunk_rows:
            btree = self._write_chunk_btree(d)
            row_elems = int(np.prod(d.shape[1:])) if len(d.shape) > 1 else 1
            cdims = (d.chunk_rows,) + tuple(d.shape[1:]) + (d.dtype.itemsize,)
            layout = struct.pack("<BBB", 3, 2, len(cdims)) + struct.pack("<Q", btree) + \
                struct.pack("<%dI" % len(cdims), *cdims)
            msgs = [
                (0x0001, _space_msg(d.shape, (None,) + tuple(d.shape[1:]))),
                (0x0003, _dtype_msg(d.dtype)),
                (0x0005, bytes([2, 3, 2, 0])),  # fill value v2: alloc incremental (3, as h5py for chunked), write if set, undefined
                (0x0008, layout),
            ]
            if d.compression == "lzf":
                msgs.append((0x000B, _lzf_filter_msg(d.chunk_rows * row_elems * d.dtype.itemsize)))
            for k, v in d.attrs.items():
                msgs.append((0x000C, self._attr_msg(k, v)))
            return self._object_header(msgs)
        if d.data is not None:
            raw = d.data.tobytes()
            addr = self._alloc(raw) if raw else UNDEF
            nbytes = len(raw)
        else:
            addr = d.addr if d.addr is not None else UNDEF
            nbytes = int(np.prod(d.shape)) * d.dtype.itemsize
        msgs = [
            (0x0001, _space_msg(d.shape)),
            (0x0003, _dtype_msg(d.dtype)),
            (0x0005, bytes([2, 1, 2, 0])),  # fill value v2: alloc early, write never, undefined
            (0x0008, struct.pack("<BBQQ", 3, 1, addr, nbytes)),
        ]
        for k, v in d.attrs.items():
            msgs.append((0x000C, self._attr_msg(k, v)))
        return self._object_header(msgs)

    def _write_group(self, g: _WGroup) -> Tuple[int, int, int]:
        # children first
        entries = []
        for name, ch in g.children.items():
            if isinstance(ch, _WGroup):
                oh, bt, hp = self._write_group(ch)
                entries.append((name.encode("utf-8"), oh, (bt, hp)))
            else:
                entries.append((name.encode("utf-8"), self._write_dataset(ch), None))
        entries.sort(key=lambda e: e[0])
        # local heap: "" at offset 0, then names
        heap = bytearray(b"\0" * 8)
        name_off = []
        for nm, _, _ in entries:
            name_off.append(len(heap))
            heap += nm + b"\0"
            heap += b"\0" * (_pad8(len(heap)) - len(heap))
        heap += b"\0" * 8  # keep a little free space
        heap_data = self._alloc(bytes(heap))
        heap_addr = self._alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap), UNDEF, heap_data))
        # symbol nodes
        cap = 2 * self.LEAF_K
        snods = []  # (addr, max name offset)
        for i in range(0, max(1, len(entries)), cap):
            chunk = entries[i:i + cap]
            b = b"SNOD" + struct.pack("<BBH", 1, 0, len(chunk))
            for j, (nm, oh, scratch) in enumerate(chunk):
                if scratch is not None:
                    b += struct.pack("<QQII", name_off[i + j], oh, 1, 0) + struct.pack("<QQ", *scratch)
                else:
                    b += struct.pack("<QQII", name_off[i + j], oh, 0, 0) + b"\0" * 16
            b += b"\0" * (40 * (cap - len(chunk)))
            snods.append((self._alloc(b), name_off[i + len(chunk) - 1] if chunk else 0))
        btree = self._write_btree(snods, 0)
        msgs = [(0x0011, struct.pack("<QQ", btree, heap_addr))]
        for k, v in g.attrs.items():
            msgs.append((0x000C, self._attr_msg(k, v)))
        oh = self._object_header(msgs)
        return oh, btree, heap_addr

    def _write_btree(self, children: List[Tuple[int, int]], level: int) -> int:
        cap = 2 * self.INTERNAL_K
        nodes = []
        groups = [children[i:i + cap] for i in range(0, len(children), cap)]
        size = 24 + (cap + 1) * 8 + cap * 8
        base = self._tell()
        addrs = [base + k * _pad8(size) for k in range(len(groups))]
        for k, grp in enumerate(groups):
            left = addrs[k - 1] if k > 0 else UNDEF
            right = addrs[k + 1] if k + 1 < len(groups) else UNDEF
            b = b"TREE" + struct.pack("<BBHQQ", 0, level, len(grp), left, right)
            b += struct.pack("<Q", 0)
            for caddr, maxoff in grp:
                b += struct.pack("<QQ", caddr, maxoff)
            b += b"\0" * (size - len(b))
            a = self._alloc(b)
            assert a == addrs[k]
            nodes.append((a, grp[-1][1]))
        if len(nodes) == 1:
            return nodes[0][0]
        return self._write_btree(nodes, level + 1)

    def close(self) -> None:
        if self._closed:
            return
        if self._stream_open is not None:
            self._stream_open.finish()
        self._fh.seek(0, io.SEEK_END)
        pad = _pad8(self._tell()) - self._tell()
        self._fh.write(b"\0" * pad)
        root_oh, root_bt, root_hp = self._write_group(self)
        eof = self._tell()
        sb = SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", self.LEAF_K, self.INTERNAL_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, root_oh, 1, 0) + struct.pack("<QQ", root_bt, root_hp)
        assert len(sb) == 96
        self._fh.seek(0)
        self._fh.write(sb)
        self._fh.close()
        self._closed = True

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        self.close()
