"""Read-only HDF5 subset, enough for Keras weight files (no h5py in this stack).

The reference loads ``audioModel.keras`` with ``tf.keras.models.load_model``
(src/identify_tracks.py:302-327); a ``.keras`` file is a zip whose
``model.weights.h5`` holds the weights as HDF5 datasets.  This module reads
what the HDF5 library writes for such files:

* superblock versions 0-3 (8-byte offsets and lengths);
* object headers version 1 and 2 (with continuation blocks);
* groups in both storage forms: symbol tables (B-tree v1 + local heap, the
  default of h5py/libver "earliest") and compact link messages (newer
  libver); dense link storage (fractal heap) is rejected;
* datasets with compact or contiguous layout (layout message v3 / v4) or
  chunked layout with a B-tree v1 index (v3, unfiltered), of little- or
  big-endian IEEE floats (2/4/8 bytes) and integers.

Anything else raises ``ValueError``.  Pinned by tests/golden/h5/, files written
by the real HDF5 library (h5py 3.3 / HDF5 1.12) with tests/golden/make_h5.py.
"""
from __future__ import annotations

import struct

import numpy as np

_SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class H5File:
    def __init__(self, data: bytes):
        self.d = data
        base = None
        for off in (0, 512, 1024, 2048, 4096, 8192):
            if data[off:off + 8] == _SIG:
                base = off
                break
        if base is None:
            raise ValueError("not an HDF5 file")
        ver = data[base + 8]
        if ver in (0, 1):
            so, sl = data[base + 13], data[base + 14]
            if (so, sl) != (8, 8):
                raise ValueError(f"HDF5 offset/length sizes {so}/{sl} unsupported")
            p = base + 24 + (4 if ver == 1 else 0)
            self.base = self._u(p, 8)
            # root group symbol table entry: after base, free-space, EOF, driver addresses
            entry = p + 32
            self.root = self._u(entry + 8, 8)
        elif ver in (2, 3):
            so, sl = data[base + 9], data[base + 10]
            if (so, sl) != (8, 8):
                raise ValueError(f"HDF5 offset/length sizes {so}/{sl} unsupported")
            self.base = self._u(base + 12, 8)
            self.root = self._u(base + 12 + 24, 8)
        else:
            raise ValueError(f"HDF5 superblock version {ver} unsupported")

    # ---- primitives ----
    def _u(self, p, n):
        return int.from_bytes(self.d[p:p + n], "little")

    def _a(self, addr):  # file offset of an address
        return self.base + addr

    # ---- object headers ----
    def messages(self, addr):
        """[(type, body bytes)] of the object header at ``addr``."""
        p = self._a(addr)
        out = []
        if self.d[p:p + 4] == b"OHDR":
            ver, flags = self.d[p + 4], self.d[p + 5]
            q = p + 6
            if flags & 0x20:
                q += 16  # access / modification / change / birth times
            if flags & 0x10:
                q += 4  # max compact / min dense attributes
            nsz = 1 << (flags & 3)
            size = self._u(q, nsz)
            q += nsz
            self._msgs_v2(q, size, flags, out)
        else:
            if self.d[p] != 1:
                raise ValueError(f"object header version {self.d[p]} unsupported")
            nmsg = self._u(p + 2, 2)
            size = self._u(p + 8, 4)
            self._msgs_v1(p + 16, size, out, nmsg)
        return out

    def _msgs_v1(self, q, size, out, nmsg):
        end = q + size
        while q + 8 <= end:
            t, sz = self._u(q, 2), self._u(q + 2, 2)
            body = self.d[q + 8:q + 8 + sz]
            if t == 0x10:  # continuation
                a, ln = struct.unpack("<QQ", body[:16])
                self._msgs_v1(self._a(a), ln, out, nmsg)
            else:
                out.append((t, body))
            q += 8 + sz

    def _msgs_v2(self, q, size, flags, out):
        end = q + size
        while q + 4 <= end:
            t, sz = self.d[q], self._u(q + 1, 2)
            mflags = self.d[q + 3]
            h = 4 + (2 if flags & 0x04 else 0)
            body = self.d[q + h:q + h + sz]
            if t == 0x10:
                a, ln = struct.unpack("<QQ", body[:16])
                c = self._a(a)
                if self.d[c:c + 4] != b"OCHK":
                    raise ValueError("bad continuation block")
                self._msgs_v2(c + 4, ln - 8, flags, out)  # minus signature and checksum
            elif t != 0:
                out.append((t, body))
            q += h + sz
            del mflags

    # ---- groups ----
    def children(self, addr):
        """{name: object header address} of the group at ``addr``."""
        res = {}
        for t, b in self.messages(addr):
            if t == 0x11:  # symbol table: B-tree v1 + local heap
                btree, heap = struct.unpack("<QQ", b[:16])
                self._symtab(btree, self._heap_data(heap), res)
            elif t == 0x06:  # link message (compact storage)
                name, target = self._link(b)
                if target is not None:
                    res[name] = target
            elif t == 0x02:  # link info
                fheap = struct.unpack("<Q", b[2 + (8 if b[1] & 1 else 0):][:8])[0]
                if fheap != UNDEF:
                    raise ValueError("dense link storage (fractal heap) unsupported")
        return res

    def _heap_data(self, addr):
        p = self._a(addr)
        if self.d[p:p + 4] != b"HEAP":
            raise ValueError("bad local heap")
        return self._a(self._u(p + 24, 8))

    def _cstr(self, p):
        e = self.d.index(b"\0", p)
        return self.d[p:e].decode()

    def _symtab(self, btree, heap, res):
        p = self._a(btree)
        if self.d[p:p + 4] != b"TREE" or self.d[p + 4] != 0:
            raise ValueError("bad group B-tree")
        level, n = self.d[p + 5], self._u(p + 6, 2)
        q = p + 24  # signature, type, level, entries, left, right
        q += 8  # key 0
        for _ in range(n):
            child = self._u(q, 8)
            q += 16  # child + next key
            if level > 0:
                self._symtab(child, heap, res)
                continue
            s = self._a(child)
            if self.d[s:s + 4] != b"SNOD":
                raise ValueError("bad symbol table node")
            for k in range(self._u(s + 6, 2)):
                e = s + 8 + 40 * k
                res[self._cstr(heap + self._u(e, 8))] = self._u(e + 8, 8)

    def _link(self, b):
        ver, flags = b[0], b[1]
        q = 2
        ltype = 0
        if flags & 0x08:
            ltype = b[q]
            q += 1
        if flags & 0x04:
            q += 8
        if flags & 0x10:
            q += 1
        nsz = 1 << (flags & 3)
        ln = int.from_bytes(b[q:q + nsz], "little")
        q += nsz
        name = b[q:q + ln].decode()
        q += ln
        if ltype != 0:  # soft / external links are not followed
            return name, None
        return name, int.from_bytes(b[q:q + 8], "little")

    def get(self, path):
        addr = self.root
        for part in [x for x in path.split("/") if x]:
            kids = self.children(addr)
            if part not in kids:
                raise KeyError(path)
            addr = kids[part]
        return addr

    def keys(self, path=""):
        return list(self.children(self.get(path)).keys())

    def is_dataset(self, addr):
        return any(t == 0x08 for t, _ in self.messages(addr))

    # ---- datasets ----
    def read(self, path_or_addr) -> np.ndarray:
        addr = self.get(path_or_addr) if isinstance(path_or_addr, str) else path_or_addr
        shape = dtype = layout = None
        for t, b in self.messages(addr):
            if t == 0x01:
                shape = self._dataspace(b)
            elif t == 0x03:
                dtype = self._datatype(b)
            elif t == 0x08:
                layout = b
            elif t == 0x0B:
                raise ValueError("filtered (compressed) datasets unsupported")
        if shape is None or dtype is None or layout is None:
            raise ValueError("not a dataset")
        n = int(np.prod(shape)) if shape else 1
        ver = layout[0]
        if ver not in (3, 4):
            raise ValueError(f"data layout version {ver} unsupported")
        cls = layout[1]
        if ver == 4 and cls == 2:
            raise ValueError("chunked layout v4 (libver latest chunk indexes) unsupported")
        if cls == 0:  # compact
            sz = int.from_bytes(layout[2:4], "little")
            raw = layout[4:4 + sz]
        elif cls == 1:  # contiguous
            a, sz = struct.unpack("<QQ", layout[2:18])
            if a == UNDEF:  # never written: the fill value (0)
                return np.zeros(shape, dtype.newbyteorder("="))
            raw = self.d[self._a(a):self._a(a) + sz]
        elif cls == 2:  # chunked
            return self._chunked(layout, shape, dtype)
        else:
            raise ValueError(f"layout class {cls} unsupported")
        return np.frombuffer(raw[:n * dtype.itemsize], dtype).reshape(shape).astype(dtype.newbyteorder("="))

    def _dataspace(self, b):
        ver, rank, flags = b[0], b[1], b[2]
        q = 8 if ver == 1 else 4
        if ver == 2 and b[3] == 0:  # scalar
            return ()
        dims = [int.from_bytes(b[q + 8 * i:q + 8 * i + 8], "little") for i in range(rank)]
        return tuple(dims)

    def _datatype(self, b):
        cls, bits0 = b[0] & 0x0F, b[1]
        size = int.from_bytes(b[4:8], "little")
        big = bool(bits0 & 1)
        e = ">" if big else "<"
        if cls == 1:
            if size not in (2, 4, 8):
                raise ValueError(f"float size {size}")
            return np.dtype(f"{e}f{size}")
        if cls == 0:
            signed = bool(bits0 & 0x08)
            return np.dtype(f"{e}{'i' if signed else 'u'}{size}")
        raise ValueError(f"datatype class {cls} unsupported")

    def _chunked(self, layout, shape, dtype):
        rank = layout[2]  # dimensionality + 1 (last: element size)
        btree = struct.unpack("<Q", layout[3:11])[0]
        cdims = [int.from_bytes(layout[11 + 4 * i:15 + 4 * i], "little") for i in range(rank)]
        cshape = cdims[:-1]
        out = np.zeros(shape, dtype.newbyteorder("="))
        if btree == UNDEF:
            return out
        self._chunks(btree, rank, cshape, dtype, out)
        return out

    def _chunks(self, addr, rank, cshape, dtype, out):
        p = self._a(addr)
        if self.d[p:p + 4] != b"TREE" or self.d[p + 4] != 1:
            raise ValueError("bad chunk B-tree")
        level, n = self.d[p + 5], self._u(p + 6, 2)
        q = p + 24
        ksz = 8 + 8 * rank
        for i in range(n):
            key = q + i * (ksz + 8)
            csize, fmask = self._u(key, 4), self._u(key + 4, 4)
            offs = [self._u(key + 8 + 8 * j, 8) for j in range(rank - 1)]
            child = self._u(key + ksz, 8)
            if level > 0:
                self._chunks(child, rank, cshape, dtype, out)
                continue
            if fmask:
                raise ValueError("filtered chunk")
            cnt = int(np.prod(cshape))
            raw = np.frombuffer(self.d[self._a(child):self._a(child) + cnt * dtype.itemsize], dtype)
            blk = raw.reshape(cshape).astype(dtype.newbyteorder("="))
            sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cshape, out.shape))
            out[sl] = blk[tuple(slice(0, x.stop - x.start) for x in sl)]


def open_h5(path_or_bytes) -> H5File:
    if isinstance(path_or_bytes, (bytes, bytearray)):
        return H5File(bytes(path_or_bytes))
    with open(path_or_bytes, "rb") as f:
        return H5File(f.read())
