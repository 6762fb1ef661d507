"""Test-side Ogg Vorbis encoder: writes the streams the Vorbis tests decode.

It restates the encoder half of the Xiph "Vorbis I specification" for the
features the decoder must handle -- it is not a perceptual encoder:

- codebooks with ordered / sparse / plain length lists, lookup types 1 and 2,
  sequence_p, codewords assigned by the spec's lowest-free rule (3.2.1);
- floor 1 (partition classes with master books and "no book" subclasses;
  post amplitudes from the block's spectrum, coded through the spec's
  prediction / room folding, 7.2.4) and floor 0 (LSP, 6);
- residues 0, 1 and 2 with a classbook, a silent class and two-pass cascades
  (coarse + fine VQ) (8.6);
- mapping 0 with submaps and square-polar coupling (4.3.5 inverted);
- short / long blocks with window-shape flags, forward MDCT scaled 4/N so the
  unscaled inverse of 4.3.7 reconstructs the input;
- Ogg pages with CRC-32, lacing across pages, several packets per page,
  granule positions (end trim; optional start trim), an optional second
  logical stream interleaved.

Curves are computed with oracle/vorbis_oracle.py's floor functions, so the
residue the stream carries is exactly the spectrum over the curve the decoder
will rebuild.  Used by tests/test_vorbis.py only.
"""
from __future__ import annotations

import math
import struct
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from oracle import vorbis_oracle as vo  # noqa: E402


class BitWriter:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, val, bits):
        if bits:
            self.v |= (int(val) & ((1 << bits) - 1)) << self.n
            self.n += bits

    def data(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def float32_pack(x):  # inverse of Vorbis I 9.2.2 (exact for <= 21 significant bits)
    if x == 0:
        return 0
    sign = 1 if x < 0 else 0
    m, e = math.frexp(abs(x))
    mant = int(round(m * (1 << 21)))
    exp = e - 21 + 788
    if mant == 1 << 21:
        mant >>= 1
        exp += 1
    assert 0 <= exp < 1024 and mant < 1 << 21
    return sign << 31 | exp << 21 | mant


def complete_lengths(n, order=None):
    """Kraft-complete code lengths for n entries: 2^L - n entries of length
    L-1, the rest L; ``order`` lists the entries taking the short codes first."""
    L = max(1, math.ceil(math.log2(n)))
    short = (1 << L) - n
    order = list(range(n)) if order is None else list(order)
    out = [L] * n
    for e in order[:short]:
        out[e] = L - 1
    return out


class Book:
    def __init__(self, lengths, dims=1, lookup=0, minv=0.0, delta=1.0, vbits=1, seq=0, mults=None,
                 ordered=False, sparse=False):
        self.lengths, self.dims, self.lookup = list(lengths), dims, lookup
        self.minv, self.delta, self.vbits, self.seq, self.mults = minv, delta, vbits, seq, mults
        self.ordered, self.sparse = ordered, sparse
        if ordered:
            assert all(a <= b for a, b in zip(self.lengths, self.lengths[1:])) and 0 not in self.lengths
        taken, self.codes = [], {}
        for e, ln in enumerate(self.lengths):
            if ln:
                c = vo.Codebook._lowest_free(ln, taken)
                assert c is not None
                self.codes[e] = c
        self.used = np.array([ln > 0 for ln in self.lengths])
        if lookup:
            self.vq = self._vectors()

    def _vectors(self):
        E, D = len(self.lengths), self.dims
        nval = vo.lookup1_values(E, D) if self.lookup == 1 else E * D
        assert len(self.mults) == nval
        mn, dl = np.float32(vo.float32_unpack(float32_pack(self.minv))), vo.float32_unpack(float32_pack(self.delta))
        vq = np.zeros((E, D), np.float32)
        for e in range(E):
            last, div = np.float32(0), 1
            for i in range(D):
                off = (e // div) % nval if self.lookup == 1 else e * D + i
                v = np.float32(np.float32(self.mults[off]) * dl + mn + last)
                vq[e, i] = v
                if self.seq:
                    last = v
                if self.lookup == 1:
                    div *= nval
        return vq

    def header(self, bw):
        E = len(self.lengths)
        bw.put(0x564342, 24)
        bw.put(self.dims, 16)
        bw.put(E, 24)
        bw.put(1 if self.ordered else 0, 1)
        if self.ordered:
            cur, ln = 0, self.lengths[0]
            bw.put(ln - 1, 5)
            while cur < E:
                num = sum(1 for x in self.lengths[cur:] if x == ln)
                bw.put(num, vo.ilog(E - cur))
                cur += num
                ln += 1
        else:
            bw.put(1 if self.sparse else 0, 1)
            for ln in self.lengths:
                if self.sparse:
                    bw.put(1 if ln else 0, 1)
                    if not ln:
                        continue
                bw.put(ln - 1, 5)
        bw.put(self.lookup, 4)
        if self.lookup:
            bw.put(float32_pack(self.minv), 32)
            bw.put(float32_pack(self.delta), 32)
            bw.put(self.vbits - 1, 4)
            bw.put(self.seq, 1)
            for m in self.mults:
                bw.put(m, self.vbits)

    def put(self, bw, e):
        for ch in self.codes[int(e)]:  # first bit read = first character
            bw.put(1 if ch == "1" else 0, 1)

    def nearest(self, vecs):
        """Index of the used entry nearest each row of vecs [k, dims]."""
        d = ((vecs[:, None, :] - self.vq[None, :, :]) ** 2).sum(-1)
        d[:, ~self.used] = np.inf
        return d.argmin(1)


# --------------------------------------------------------------------- books
def scalar_book(n, order=None, **kw):
    return Book(complete_lengths(n, order), **kw)


def coarse_book(lim=15, seq=0, sparse=False):
    """dims 2, lookup 1: values -lim..lim per dimension (seq: v1 += v0)."""
    r = 2 * lim + 1
    n = r * r
    center = (n - 1) // 2
    order = sorted(range(n), key=lambda e: abs(e - center))  # short codes near zero
    if sparse:  # two corner entries unused; the used ones form a complete code
        used = [e for e in range(n) if e not in (0, n - 1)]
        sub = complete_lengths(len(used), [used.index(e) for e in order if e in used])
        lengths = [0] * n
        for e, ln in zip(used, sub):
            lengths[e] = ln
    else:
        lengths = complete_lengths(n, order)
    return Book(lengths, dims=2, lookup=1, minv=-float(lim), delta=1.0, vbits=5, seq=seq,
                mults=list(range(r)), sparse=sparse)


def fine_book():
    """dims 2, lookup 2: the grid -0.5..0.5 step 0.125 per dimension."""
    grid = [(a, b) for a in range(9) for b in range(9)]
    return Book(complete_lengths(81), dims=2, lookup=2, minv=-0.5, delta=0.125, vbits=4,
                mults=[m for ab in grid for m in ab])


def lsp_book():
    """dims 2, lookup 1, values 0.2..3.0 (floor 0 LSP coefficient pairs, seq)."""
    return Book(complete_lengths(225), dims=2, lookup=1, minv=0.2, delta=0.2, vbits=4, seq=1,
                mults=list(range(15)))


# ---------------------------------------------------------------- floor 1 cfg
class Floor1Cfg:
    """Posts: 0, n2 and a log-spaced set; partitions alternate class 0 (dim 3,
    one subclass bit: Y book or no book, with a master book) and class 1
    (dim 2, no subclass bits)."""

    def __init__(self, n2, ybook, master, mult=2):
        self.n2, self.mult, self.rng = n2, mult, vo.Floor1.RANGES[mult - 1]
        self.rb = int(math.log2(n2))
        assert 1 << self.rb == n2
        posts = sorted({int(round(v)) for v in np.geomspace(2, n2 - 1, min(40, n2 // 3))} - {0, n2})
        self.classes = [(3, 1), (2, 0)]
        self.part_class, xs, i = [], [], 0
        while i < len(posts):
            c = len(self.part_class) % 2
            d = self.classes[c][0]
            if i + d > len(posts):
                c, d = 1, 2
                if i + d > len(posts):
                    break
            self.part_class.append(c)
            xs += posts[i:i + d]
            i += d
        self.X = [0, n2] + xs
        self.ybook, self.master = ybook, master

    def header(self, bw, ybook_id, master_id):
        bw.put(1, 16)
        bw.put(len(self.part_class), 5)
        for c in self.part_class:
            bw.put(c, 4)
        for d, sub in self.classes:
            bw.put(d - 1, 3)
            bw.put(sub, 2)
            if sub:
                bw.put(master_id, 8)
            books = [ybook_id, -1] if sub else [ybook_id]
            for b in books:
                bw.put(b + 1, 8)
        bw.put(self.mult - 1, 2)
        bw.put(self.rb, 4)
        for x in self.X[2:]:
            bw.put(x, self.rb)

    def oracle(self):
        f = vo.Floor1.__new__(vo.Floor1)
        f.X, f.mult = self.X, self.mult
        return f

    def _vals(self, target):
        """Stream values coding the target post amplitudes: the first two raw,
        the rest through the prediction folding of 7.2.4 step 1 (the val
        reproducing each target found by scanning the folding)."""
        X, rng = self.X, self.rng
        vals, fy = [target[0], target[1]], [target[0], target[1]]
        for i in range(2, len(X)):
            lo, hi = vo.Floor1.neighbours(X, i)
            dy, adx = fy[hi] - fy[lo], X[hi] - X[lo]
            off = abs(dy) * (X[i] - X[lo]) // adx
            pred = fy[lo] - off if dy < 0 else fy[lo] + off
            highroom, lowroom = rng - pred, pred
            room = min(highroom, lowroom) * 2
            best, got = 0, pred
            if target[i] != pred:
                for v in range(1, rng):
                    if v >= room:
                        y = v - lowroom + pred if highroom > lowroom else pred - v + highroom - 1
                    else:
                        y = pred - (v + 1) // 2 if v & 1 else pred + v // 2
                    if y == target[i]:
                        best, got = v, y
                        break
            vals.append(best)
            fy.append(got)
        return vals, fy

    def encode(self, bw, spec, headroom=4.0):
        """Choose post amplitudes for |spec| (None: unused floor), write them,
        return the curve the decoder will build."""
        if spec is None:
            bw.put(0, 1)
            return None
        f = self.oracle()
        A = np.abs(spec)
        # target Y per post: the level at which |spec| near the post is <= headroom x curve
        X = self.X
        xs = sorted(X)
        target = []
        for x in X:
            k = xs.index(x)
            lo = xs[k - 1] if k > 0 else 0
            hi = xs[k + 1] if k + 1 < len(xs) else self.n2
            a = float(A[max(0, (lo + x) // 2):max(min(self.n2, (x + hi) // 2 + 1), 1)].max(initial=0.0))
            want = max(a / headroom, 1e-7)
            y = int(np.searchsorted(vo.INV_DB[::self.mult][:self.rng], want))
            target.append(min(max(y, 0), self.rng - 1))
        # raise posts until the curve covers the spectrum within the residue
        # books' range everywhere (the curve is linear in dB between posts)
        order = sorted(range(len(X)), key=lambda i: X[i])
        for _ in range(64):
            vals, fy = self._vals(target)
            curve = f.curve(*f.final_y(vals), self.n2)
            over = False
            for a, b in zip(order, order[1:]):
                seg = slice(X[a], min(X[b] + 1, self.n2))
                if float(np.max(A[seg] / curve[seg], initial=0.0)) > 6.0:
                    for i in (a, b):
                        if target[i] < self.rng - 1:
                            target[i] += 1
                            over = True
            if not over:
                break
        vals, fy = self._vals(target)
        bw.put(1, 1)
        bits = vo.ilog(self.rng - 1)
        bw.put(vals[0], bits)
        bw.put(vals[1], bits)
        off = 2
        for c in self.part_class:
            d, sub = self.classes[c]
            if sub:
                cval = 0
                for j in range(d):
                    if vals[off + j] == 0:
                        cval |= 1 << j  # subclass 1: no book, Y = 0
                self.master.put(bw, cval)
                for j in range(d):
                    if not (cval >> j) & 1:
                        self.ybook.put(bw, vals[off + j])
            else:
                for j in range(d):
                    self.ybook.put(bw, vals[off + j])
            off += d
        fy, step2 = f.final_y(vals)
        return f.curve(fy, step2, self.n2)


# ---------------------------------------------------------------- floor 0 cfg
class Floor0Cfg:
    def __init__(self, rate, book, order=4, bark_size=128, amp_bits=8, amp_offset=140):
        self.rate, self.book, self.order = rate, book, order
        self.bark_size, self.amp_bits, self.amp_offset = bark_size, amp_bits, amp_offset
        self.coef_entries = [7 * 15 + 3, 2 * 15 + 4]  # LSP pairs (seq: second value adds the first)

    def header(self, bw, book_id):
        bw.put(0, 16)
        bw.put(self.order, 8)
        bw.put(self.rate, 16)
        bw.put(self.bark_size, 16)
        bw.put(self.amp_bits, 6)
        bw.put(self.amp_offset, 8)
        bw.put(0, 4)  # one book
        bw.put(book_id, 8)

    def oracle(self):
        f = vo.Floor0.__new__(vo.Floor0)
        f.order, f.rate, f.bark_size, f.amp_bits, f.amp_offset = (self.order, self.rate, self.bark_size,
                                                                 self.amp_bits, self.amp_offset)
        return f

    def coef(self, entries=None):
        out, last = [], np.float32(0)
        for e in (entries or self.coef_entries):
            for v in self.book.vq[e]:
                out.append(np.float32(v + last))
            last = out[-1]
        return out[:self.order]

    def _pq_np(self, coef, n2):
        """Vectorised sqrt(p + q) of 6.2.3 (the search's estimate; the residue
        uses the oracle's curve)."""
        i = np.arange(n2)
        bark = lambda x: 13.1 * np.arctan(.00074 * x) + 2.24 * np.arctan(.0000000185 * x * x) + .0001 * x
        mp = np.minimum(self.bark_size - 1, np.floor(bark(self.rate * i / (2.0 * n2)) * self.bark_size
                                                    / bark(0.5 * self.rate)))
        cw = np.cos(np.pi * mp / self.bark_size)
        cc = np.cos(np.asarray(coef, np.float64))
        p = (1.0 - cw) / 2.0 * np.prod([4.0 * (cc[j] - cw) ** 2 for j in range(1, self.order, 2)], 0)
        q = (1.0 + cw) / 2.0 * np.prod([4.0 * (cc[j] - cw) ** 2 for j in range(0, self.order, 2)], 0)
        return np.sqrt(p + q)

    def encode(self, bw, spec, n2, headroom=6.0):
        if spec is None:
            bw.put(0, self.amp_bits)
            return None
        assert self.order % 2 == 0
        A = np.abs(spec).astype(np.float64)
        amax = (1 << self.amp_bits) - 1
        amps = np.arange(1, amax + 1, dtype=np.float64)[:, None]
        best = None
        # LSP pairs and amplitude minimising the expected error: the spectrum
        # the residue books cannot reach (|r| > 7) plus the fine grid's
        # quantisation noise (rms 0.036 of the curve)
        for e1 in range(0, 225, 8):
            for e2 in range(3, 225, 8):
                coef = self.coef([e1, e2])
                with np.errstate(over="ignore", divide="ignore", invalid="ignore"):
                    db = amps * self.amp_offset / amax / self._pq_np(coef, n2)[None, :] - self.amp_offset
                    curve = np.exp(0.11512925 * np.minimum(db, 80.0))
                    err = (np.maximum(A[None, :] - 7.0 * curve, 0.0) ** 2 + (0.036 * curve) ** 2).sum(1)
                k = int(np.nanargmin(err))
                if best is None or err[k] < best[0]:
                    best = (err[k], [e1, e2], k + 1)
        _, self.coef_entries, amp = best
        f, coef = self.oracle(), self.coef()
        c = f.curve(amp, coef, n2)
        bw.put(amp, self.amp_bits)
        bw.put(0, vo.ilog(1))  # book number 0 of 1
        for e in self.coef_entries:
            self.book.put(bw, e)
        return c


# ------------------------------------------------------------------ residues
class ResidueCfg:
    """Partitions of ``psize`` over [0, end); class 0 silent, class 1 coarse +
    fine, class 2 a sequence_p coarse book + fine; classbook dims 2."""

    def __init__(self, rtype, psize, end, classbook, coarse, coarse_seq, fine, begin=0):
        self.type, self.psize, self.end, self.begin = rtype, psize, end, begin
        self.classbook, self.books = classbook, {1: [coarse, fine], 2: [coarse_seq, fine]}
        self.classes = 3

    def header(self, bw, ids):
        bw.put(self.type, 16)
        bw.put(self.begin, 24)
        bw.put(self.end, 24)
        bw.put(self.psize - 1, 24)
        bw.put(self.classes - 1, 6)
        bw.put(ids[self.classbook], 8)
        casc = [0, 0b11, 0b11]
        for c in casc:
            bw.put(c & 7, 3)
            bw.put(0, 1)
        for c in range(self.classes):
            for p in range(8):
                if casc[c] & (1 << p):
                    bw.put(ids[self.books[c][p]], 8)

    def _vectors(self, seg, book, fmt):
        """Rows of the partition as the decoder adds them (format 0 interleaves)."""
        d = book.dims
        if fmt == 0:
            step = len(seg) // d
            return np.stack([seg[s::step][:d] for s in range(step)])
        return seg.reshape(-1, d)

    def _unvectors(self, vecs, n, fmt):
        d = vecs.shape[1]
        if fmt == 0:
            step = n // d
            out = np.zeros(n, np.float32)
            for s in range(step):
                out[s::step][:d] = vecs[s]
            return out
        return vecs.reshape(-1)[:n]

    def encode(self, bw, vecs, dnd, n, fmt):
        """Quantise and write residue vectors (each [n], float32); returns what
        the decoder will reconstruct."""
        lb, le = min(self.begin, n), min(self.end, n)
        nparts = (le - lb) // self.psize
        cpw = self.classbook.dims
        out = [np.zeros(n, np.float32) for _ in vecs]
        if nparts <= 0:
            return out
        cls = []
        for j, v in enumerate(vecs):
            cj = []
            for p in range(nparts):
                seg = v[lb + p * self.psize:lb + (p + 1) * self.psize]
                cj.append(0 if np.abs(seg).max() < 0.0625 else (1 if p % 3 else 2))
            cls.append(cj + [0] * cpw)
        # quantise every non-silent partition: pass 0 coarse, pass 1 fine
        q = {}
        for j, v in enumerate(vecs):
            if dnd[j]:
                continue
            for p in range(nparts):
                c = cls[j][p]
                if c == 0:
                    continue
                seg = v[lb + p * self.psize:lb + (p + 1) * self.psize].astype(np.float32)
                coarse, fine = self.books[c]
                e0 = coarse.nearest(self._vectors(seg, coarse, fmt))
                r0 = self._unvectors(coarse.vq[e0], self.psize, fmt)
                e1 = fine.nearest(self._vectors((seg - r0).astype(np.float32), fine, fmt))
                r1 = self._unvectors(fine.vq[e1], self.psize, fmt)
                q[(j, p)] = (e0, e1)
                out[j][lb + p * self.psize:lb + (p + 1) * self.psize] = (r0 + r1).astype(np.float32)
        for pas in range(2):
            pc = 0
            while pc < nparts:
                if pas == 0:
                    for j in range(len(vecs)):
                        if dnd[j]:
                            continue
                        t = 0
                        for i in range(cpw):
                            t = t * self.classes + cls[j][pc + i]
                        self.classbook.put(bw, t)
                i = 0
                while i < cpw and pc < nparts:
                    for j in range(len(vecs)):
                        if dnd[j] or cls[j][pc] == 0:
                            continue
                        book = self.books[cls[j][pc]][pas]
                        for e in q[(j, pc)][pas]:
                            book.put(bw, e)
                    i += 1
                    pc += 1
        return out


def couple(x, y):
    """Square-polar forward coupling: (magnitude, angle) whose inverse
    (Vorbis I 4.3.5) returns (x, y)."""
    M, A = np.empty_like(x), np.empty_like(x)
    for j in range(len(x)):
        a, b = x[j], y[j]
        if a > 0:
            M[j], A[j] = (a, a - b) if b < a else (b, a - b)
        else:
            M[j], A[j] = (a, b - a) if b > a else (b, b - a)
    return M, A


def uncouple(M, A):
    M, A = M.copy(), A.copy()
    for j in range(len(M)):
        m0, a0 = M[j], A[j]
        if m0 > 0:
            M[j], A[j] = (m0, m0 - a0) if a0 > 0 else (m0 + a0, m0)
        else:
            M[j], A[j] = (m0, m0 + a0) if a0 > 0 else (m0 - a0, m0)
    return M, A


# ---------------------------------------------------------------------- Ogg
def ogg_page(serial, seq, granule, htype, segs, body):
    hdr = b"OggS" + bytes([0, htype]) + struct.pack("<qIII", granule, serial, seq, 0) + bytes([len(segs)]) + bytes(segs)
    page = bytearray(hdr + body)
    page[22:26] = struct.pack("<I", vo.ogg_crc(bytes(page)))
    return bytes(page)


def paginate(packets, granules, serial, max_segs=255, per_page=None):
    """Ogg pages of packets (headers each on their own page); granules[i]: the
    granule after audio packet i (None for headers).  max_segs small forces
    packets across pages; per_page groups several packets on one page."""
    pages, seq = [], 0
    # headers: page 0 = identification (BOS), page 1 = comment + setup
    groups = [[0], [1, 2]]
    rest = list(range(3, len(packets)))
    k = per_page or 1
    groups += [rest[i:i + k] for i in range(0, len(rest), k)]
    cont = False
    for gi, g in enumerate(groups):
        segs, body, done_gran = [], b"", None
        pending = []
        for i in g:
            p = packets[i]
            lace = [255] * (len(p) // 255) + [len(p) % 255]
            pending.append((i, p, lace))
        # emit pages of at most max_segs segments
        flat = []
        for i, p, lace in pending:
            off = 0
            for j, s in enumerate(lace):
                flat.append((i, s, p[off:off + s], j == len(lace) - 1))
                off += s
        while flat:
            chunk, flat = flat[:max_segs], flat[max_segs:]
            segs = [s for _, s, _, _ in chunk]
            body = b"".join(b for _, _, b, _ in chunk)
            ends = [i for i, _, _, last in chunk if last]
            gran = granules[ends[-1]] if ends and granules[ends[-1]] is not None else (0 if ends and ends[-1] < 3 else -1)
            htype = (1 if cont else 0) | (2 if seq == 0 else 0) | (4 if (gi == len(groups) - 1 and not flat) else 0)
            pages.append(ogg_page(serial, seq, gran, htype, segs, body))
            seq += 1
            cont = not chunk[-1][3]
    return pages


# ------------------------------------------------------------------ encoder
def window(n, bs0, f, pl, nl):
    return vo.window(n, bs0, f, pl, nl).astype(np.float64)


def encode(x, sr=48000, bs=(256, 2048), schedule=None, residue_type=1, coupling=True, floor0_short=False,
           submaps=False, max_segs=255, per_page=1, start_trim=0, silent=(), extra_stream=False, seed=0):
    """x: float [frames] or [frames, channels] in [-1, 1].  Returns Ogg bytes.
    schedule: block flags (1 long, 0 short), repeated to cover x; silent: block
    indices written with unused floors."""
    x = np.asarray(x, np.float64)
    if x.ndim == 1:
        x = x[:, None]
    frames, C = x.shape
    bs0, bs1 = bs
    schedule = list(schedule or [1])
    # block positions in input coordinates: block 0's centre at sample -start_trim
    flags, pos = [], []
    p, k = -bs[schedule[0]] // 2 - start_trim, 0
    while True:
        f = schedule[k % len(schedule)]
        if k:
            p += 3 * bs[flags[-1]] // 4 - bs[f] // 4
        flags.append(f)
        pos.append(p)
        if p + bs[f] // 2 >= frames:
            break
        k += 1

    books = {"ybook": scalar_book(128, order=range(0, 128, 3), sparse=True), "master": scalar_book(8, ordered=False),
             "ybook2": Book(sorted(complete_lengths(64)), ordered=True),
             "class": scalar_book(9), "coarse": coarse_book(), "coarse_seq": coarse_book(seq=1, sparse=True),
             "fine": fine_book(), "lsp": lsp_book()}
    names = list(books)
    ids = {books[n]: i for i, n in enumerate(names)}
    fl = [Floor1Cfg(bs0 // 2, books["ybook"], books["master"]), Floor1Cfg(bs1 // 2, books["ybook"], books["master"])]
    f0 = Floor0Cfg(sr, books["lsp"]) if floor0_short else None
    floors = [f0 if floor0_short else fl[0], fl[1]]
    res_types = [residue_type, 0 if submaps else residue_type]
    residues = [ResidueCfg(t, 16, bs1 // 2 * (C if t == 2 else 1), books["class"], books["coarse"],
                           books["coarse_seq"], books["fine"]) for t in res_types]

    # headers
    ident = b"\x01vorbis" + struct.pack("<IBIiii", 0, C, sr, 0, 128000, 0) + bytes(
        [int(math.log2(bs0)) | int(math.log2(bs1)) << 4, 1])
    comment = b"\x03vorbis" + struct.pack("<I", 4) + b"test" + struct.pack("<I", 0) + b"\x01"
    sw = BitWriter()
    sw.put(len(names) - 1, 8)
    for n in names:
        books[n].header(sw)
    sw.put(0, 6)
    sw.put(0, 16)
    sw.put(len(floors) - 1, 6)
    for f in floors:
        if isinstance(f, Floor0Cfg):
            f.header(sw, ids[books["lsp"]])
        else:
            f.header(sw, ids[books["ybook"]], ids[books["master"]])
    sw.put(len(residues) - 1, 6)
    for r in residues:
        r.header(sw, ids)
    # mappings: 0 for short blocks (floor 0), 1 for long (floor 1); coupling
    # and submaps as asked
    sw.put(1, 6)
    for mi in range(2):
        sw.put(0, 16)
        nsub = 2 if (submaps and C > 1) else 1
        sw.put(1 if nsub > 1 else 0, 1)
        if nsub > 1:
            sw.put(nsub - 1, 4)
        cpl = coupling and C > 1
        sw.put(1 if cpl else 0, 1)
        if cpl:
            sw.put(0, 8)
            sw.put(0, vo.ilog(C - 1))
            sw.put(1, vo.ilog(C - 1))
        sw.put(0, 2)
        if nsub > 1:
            for c in range(C):
                sw.put(c % 2, 4)
        for s in range(nsub):
            sw.put(0, 8)
            sw.put(mi, 8)                     # floor: short 0, long 1
            sw.put(s if nsub > 1 else mi % len(residues), 8)
    sw.put(1, 6)  # two modes
    for f in (0, 1):
        sw.put(f, 1)
        sw.put(0, 16)
        sw.put(0, 16)
        sw.put(f, 8)
    sw.put(1, 1)
    setup = b"\x05vorbis" + sw.data()
    packets = [ident, comment, setup]
    granules = [None, None, None]

    produced = 0
    for k, (f, p) in enumerate(zip(flags, pos)):
        n = bs[f]
        pl = flags[k - 1] if k else f
        nl = flags[k + 1] if k + 1 < len(flags) else f
        w = window(n, bs0, f, pl, nl)
        seg = np.zeros((n, C))
        a, b = max(p, 0), min(p + n, frames)
        if b > a:
            seg[a - p:b - p] = x[a:b]
        nn = np.arange(n)[:, None]
        kk = np.arange(n // 2)[None, :]
        F = np.cos(2 * np.pi / n * (nn + 0.5 + n / 4) * (kk + 0.5))
        spec = [(4.0 / n) * (F.T @ (w * seg[:, c])) for c in range(C)]
        bw = BitWriter()
        bw.put(0, 1)
        bw.put(f, 1)  # mode = block flag
        if f:
            bw.put(pl, 1)
            bw.put(nl, 1)
        fcfg = floors[f]
        curves = []
        for c in range(C):
            s = None if (k in silent) else spec[c].astype(np.float32)
            if isinstance(fcfg, Floor0Cfg):
                curves.append(fcfg.encode(bw, s, n // 2))
            else:
                curves.append(fcfg.encode(bw, s))
        res = [np.zeros(n // 2, np.float32) if cv is None else (spec[c] / cv).astype(np.float32)
               for c, cv in enumerate(curves)]
        no_res = [cv is None for cv in curves]
        cpl = coupling and C > 1
        if cpl and (not no_res[0] or not no_res[1]):
            no_res[0] = no_res[1] = False
            # couple values already on the books' grid (multiples of 1/8): the
            # magnitude / angle pair is then coded exactly and the decoder's
            # sign cases (4.3.5) cannot flip on a quantised magnitude
            q = [np.clip(np.round(r * 8.0) / 8.0, -7.5, 7.5).astype(np.float32) for r in res[:2]]
            res[0], res[1] = couple(q[0], q[1])
        nsub = 2 if (submaps and C > 1) else 1
        for s in range(nsub):
            chs = [c for c in range(C) if (c % 2 if nsub > 1 else 0) == s]
            r = residues[s if nsub > 1 else f % len(residues)]
            dnd = [no_res[c] for c in chs]
            if r.type == 2:
                if all(dnd):
                    continue
                inter = np.stack([res[c] for c in chs], 1).reshape(-1).astype(np.float32)
                r.encode(bw, [inter], [False], len(inter), 1)
            else:
                r.encode(bw, [res[c] for c in chs], dnd, n // 2, r.type)
        packets.append(bw.data())
        if k:
            produced += bs[flags[k - 1]] // 4 + n // 4
        granules.append(produced)
    # granules: the stream covers `frames` samples after the start trim
    total = frames
    granules = [g if g is None else g - start_trim for g in granules]
    granules[-1] = total
    pages = paginate(packets, granules, serial=0x1234, max_segs=max_segs, per_page=per_page)
    if extra_stream:  # a second logical stream's pages interleaved (ignored by the decoder)
        other = paginate([b"\x7fFLAC-ish", b"x" * 40, b"y" * 300] + [bytes([i]) * 50 for i in range(4)],
                         [None] * 3 + [i for i in range(4)], serial=0x9999)
        mixed = []
        for i, pg in enumerate(pages):
            mixed.append(pg)
            if i < len(other):
                mixed.append(other[i])
        pages = mixed
    return b"".join(pages)


def corrupt_page(data, index, byte=40):
    """Flip one body byte of the index-th page (its CRC no longer matches)."""
    pos, k = 0, 0
    while True:
        pos = data.index(b"OggS", pos)
        if k == index:
            b = bytearray(data)
            b[pos + byte] ^= 0x5A
            return bytes(b)
        pos += 4
        k += 1
