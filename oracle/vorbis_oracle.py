"""TEST INFRASTRUCTURE ONLY -- CPU restatement of Ogg Vorbis decoding, the
checker for libaa's aa_vorbis_decode.  Product code never imports this.

Reference call site: load_recording, src/identify_tracks.py:49-62, which
decodes every file with ffmpeg (audioread.ffdec) and converts to s16.  ffmpeg
is not in the image and the reference holds no Vorbis files, so this follows
the published Xiph "Vorbis I specification" (pinned to its 2020 text: sections
3 codebooks, 4.3 audio packet decode, 6 floor 0, 7 floor 1, 8 residues, 9
helpers, 10.1 floor 1 inverse-dB table) and RFC 3533 (Ogg pages) directly, in
plain Python with an O(N^2) inverse MDCT (the product uses an FFT).
PARITY UNPINNED against ffmpeg/libvorbis: no reference decoder or reference
stream exists here; tests pin it by round trips through tests/vorbis_writer.py.
"""
from __future__ import annotations

import bisect
import math
import struct

import numpy as np


def ilog(x):
    return int(x).bit_length() if x > 0 else 0


# ---------------------------------------------------------------- Ogg (RFC 3533)
def _crc_table():
    t = []
    for i in range(256):
        r = i << 24
        for _ in range(8):
            r = ((r << 1) ^ 0x04C11DB7) & 0xFFFFFFFF if r & 0x80000000 else (r << 1) & 0xFFFFFFFF
        t.append(r)
    return t


CRC = _crc_table()


def ogg_crc(page: bytes) -> int:
    c = 0
    for i, b in enumerate(page):
        if 22 <= i < 26:
            b = 0
        c = ((c << 8) & 0xFFFFFFFF) ^ CRC[((c >> 24) ^ b) & 0xFF]
    return c


def read_packets(data: bytes):
    """[(packet bytes, granule or -1, page index)] of the first Vorbis
    logical stream; granule set on the last packet completed on a page.
    Returns (packets, index of the last page)."""
    pos, serial, page_no, cur, in_pkt, out = 0, None, -1, b"", False, []
    while pos + 27 <= len(data):
        if data[pos:pos + 4] != b"OggS":
            pos += 1
            continue
        nseg = data[pos + 26]
        if data[pos + 4] != 0 or pos + 27 + nseg > len(data):
            pos += 1
            continue
        segs = data[pos + 27:pos + 27 + nseg]
        size = 27 + nseg + sum(segs)
        page = data[pos:pos + size]
        if len(page) < size or ogg_crc(page) != struct.unpack("<I", page[22:26])[0]:
            pos += 1
            continue
        htype = page[5]
        granule, ser = struct.unpack("<qI", page[6:18])
        body = page[27 + nseg:]
        if serial is None:
            if htype & 2 and body[:7] == b"\x01vorbis":
                serial = ser
            else:
                pos += size
                continue
        if ser != serial:
            pos += size
            continue
        page_no += 1
        if not htype & 1 and in_pkt:
            cur, in_pkt = b"", False
        j0, off = 0, 0
        if htype & 1 and not in_pkt:
            while j0 < nseg:
                off += segs[j0]
                j0 += 1
                if segs[j0 - 1] < 255:
                    break
        last = -1
        for j in range(j0, nseg):
            cur += body[off:off + segs[j]]
            off += segs[j]
            in_pkt = True
            if segs[j] < 255:
                out.append([cur, -1, page_no])
                cur, in_pkt = b"", False
                last = len(out) - 1
        if last >= 0:
            out[last][1] = granule
        pos += size
        if htype & 4:
            break
    if serial is None:
        raise ValueError("Ogg: no Vorbis stream")
    return out, page_no


# ------------------------------------------------------------------ bit reader
class Bits:
    """LSB-first bit reader (Vorbis I 2.1.4); eop set when reading past the end."""

    def __init__(self, data: bytes):
        self.v = int.from_bytes(data, "little")
        self.n = len(data) * 8
        self.pos = 0
        self.eop = False

    def get(self, k):
        if k == 0:
            return 0
        if self.pos + k > self.n:
            self.eop = True
            self.pos = self.n
            return 0
        r = (self.v >> self.pos) & ((1 << k) - 1)
        self.pos += k
        return r


def float32_unpack(x):  # Vorbis I 9.2.2
    mant = x & 0x1FFFFF
    exp = (x & 0x7FE00000) >> 21
    if x & 0x80000000:
        mant = -mant
    return np.float32(math.ldexp(mant, exp - 788))


def lookup1_values(entries, dims):
    r = int(math.floor(entries ** (1.0 / dims)))
    while r > 0 and r ** dims > entries:
        r -= 1
    while (r + 1) ** dims <= entries:
        r += 1
    return r


class Codebook:
    def __init__(self, br: Bits):
        if br.get(24) != 0x564342:
            raise ValueError("Vorbis: bad codebook sync")
        self.dims, self.entries = br.get(16), br.get(24)
        lengths = [0] * self.entries
        if not br.get(1):
            sparse = br.get(1)
            for i in range(self.entries):
                if sparse and not br.get(1):
                    continue
                lengths[i] = br.get(5) + 1
        else:
            cur, ln = 0, br.get(5) + 1
            while cur < self.entries:
                num = br.get(ilog(self.entries - cur))
                if cur + num > self.entries:
                    raise ValueError("Vorbis: bad ordered codebook")
                for i in range(num):
                    lengths[cur + i] = ln
                cur += num
                ln += 1
        self.lengths = lengths
        # codewords: each entry in order takes the lowest free codeword of its
        # length (Vorbis I 3.2.1) -- as a bit-string map
        self.codes = {}
        used = [i for i, ln in enumerate(lengths) if ln]
        self.single = used[0] if len(used) == 1 else None
        if len(used) > 1:
            taken = []  # assigned codeword intervals
            for i in used:
                c = self._lowest_free(lengths[i], taken)
                if c is None:
                    raise ValueError("Vorbis: overspecified codebook")
                self.codes[c] = i
        self.lookup = br.get(4)
        self.vq = None
        if self.lookup > 2:
            raise ValueError("Vorbis: bad lookup type")
        if self.lookup:
            mn, delta = float32_unpack(br.get(32)), float32_unpack(br.get(32))
            vbits, seq = br.get(4) + 1, br.get(1)
            nval = lookup1_values(self.entries, self.dims) if self.lookup == 1 else self.entries * self.dims
            mult = [br.get(vbits) for _ in range(nval)]
            vq = np.zeros((self.entries, self.dims), np.float32)
            for e in range(self.entries):
                last, div = np.float32(0), 1
                for i in range(self.dims):
                    off = (e // div) % nval if self.lookup == 1 else e * self.dims + i
                    v = np.float32(np.float32(mult[off]) * delta + mn + last)
                    vq[e, i] = v
                    if seq:
                        last = v
                    if self.lookup == 1:
                        div *= nval
            self.vq = vq
        if br.eop:
            raise ValueError("Vorbis: truncated codebook")

    @staticmethod
    def _lowest_free(length, taken):
        """The lowest codeword of this length (MSB first) whose dyadic interval
        [c 2^-L, (c+1) 2^-L) misses every taken one -- i.e. neither a prefix of
        nor prefixed by a taken codeword.  taken: sorted (start, end) in 2^-32
        units; the new interval is inserted."""
        if length > 32:
            return None
        unit = 1 << (32 - length)
        c = 0
        for s, e in taken:
            if e <= c:
                continue
            if c + unit <= s:
                break
            c = -(-e // unit) * unit
        if c + unit > 1 << 32:
            return None
        bisect.insort(taken, (c, c + unit))
        return format(c >> (32 - length), f"0{length}b")

    def decode(self, br: Bits):
        if self.single is not None:
            br.get(self.lengths[self.single])
            return -1 if br.eop else self.single
        s = ""
        while len(s) < 33:
            s += "1" if br.get(1) else "0"
            if br.eop:
                return -1
            e = self.codes.get(s)
            if e is not None:
                return e
        return -1


INV_DB = np.array([1.0649863e-07 ** ((255.0 - i) / 255.0) for i in range(256)], np.float32)  # Vorbis I 10.1


def render_line(x0, y0, x1, y1, v, n):  # Vorbis I 9.2.7
    dy, adx = y1 - y0, x1 - x0
    ady = abs(dy)
    base = int(dy / adx)  # C division: truncation toward zero
    sy = base - 1 if dy < 0 else base + 1
    ady -= abs(base) * adx
    y, err = y0, 0
    if x0 < n:
        v[x0] = INV_DB[min(max(y, 0), 255)]
    for x in range(x0 + 1, x1):
        err += ady
        if err >= adx:
            err -= adx
            y += sy
        else:
            y += base
        if x < n:
            v[x] = INV_DB[min(max(y, 0), 255)]


class Floor1:
    RANGES = (256, 128, 86, 64)

    def __init__(self, br, nbooks):
        parts = br.get(5)
        self.part_class = [br.get(4) for _ in range(parts)]
        maxc = max(self.part_class) if self.part_class else -1
        self.cdim, self.csub, self.cmaster, self.subbooks = [], [], [], []
        for _ in range(maxc + 1):
            self.cdim.append(br.get(3) + 1)
            self.csub.append(br.get(2))
            self.cmaster.append(br.get(8) if self.csub[-1] else 0)
            self.subbooks.append([br.get(8) - 1 for _ in range(1 << self.csub[-1])])
        self.mult = br.get(2) + 1
        rb = br.get(4)
        self.X = [0, 1 << rb]
        for c in self.part_class:
            for _ in range(self.cdim[c]):
                self.X.append(br.get(rb))
        if len(set(self.X)) != len(self.X):
            raise ValueError("Vorbis: repeated floor 1 X")

    @staticmethod
    def neighbours(X, i):
        lo = max((j for j in range(i) if X[j] < X[i]), key=lambda j: X[j])
        hi = min((j for j in range(i) if X[j] > X[i]), key=lambda j: X[j])
        return lo, hi

    def final_y(self, Y):
        """Vorbis I 7.2.4 step 1: (final Y values, step2 flags) of decoded Y."""
        rng = self.RANGES[self.mult - 1]
        X = self.X
        fy, step2 = list(Y[:2]), [True, True]
        for i in range(2, len(X)):
            lo, hi = self.neighbours(X, i)
            dy, adx = fy[hi] - fy[lo], X[hi] - X[lo]
            off = abs(dy) * (X[i] - X[lo]) // adx
            pred = fy[lo] - off if dy < 0 else fy[lo] + off
            val = Y[i]
            highroom, lowroom = rng - pred, pred
            room = min(highroom, lowroom) * 2
            if val:
                step2[lo] = step2[hi] = True
                step2.append(True)
                if val >= room:
                    fy.append(val - lowroom + pred if highroom > lowroom else pred - val + highroom - 1)
                else:
                    fy.append(pred - (val + 1) // 2 if val & 1 else pred + val // 2)
            else:
                step2.append(False)
                fy.append(pred)
        return fy, step2

    def curve(self, fy, step2, n2):
        """Vorbis I 7.2.4 step 2: the linear floor curve [n2] (f32)."""
        order = sorted(range(len(self.X)), key=lambda i: self.X[i])
        v = np.zeros(n2, np.float32)
        hx = hy = lx = 0
        ly = fy[order[0]] * self.mult
        for i in order[1:]:
            if step2[i]:
                hy, hx = fy[i] * self.mult, self.X[i]
                render_line(lx, ly, hx, hy, v, n2)
                lx, ly = hx, hy
        if hx < n2:
            render_line(hx, hy, n2, hy, v, n2)
        return v

    def decode(self, br, books, n2):
        if not br.get(1) or br.eop:
            return None
        rng = self.RANGES[self.mult - 1]
        Y = [br.get(ilog(rng - 1)), br.get(ilog(rng - 1))]
        for c in self.part_class:
            cbits = self.csub[c]
            cval = 0
            if cbits:
                cval = books[self.cmaster[c]].decode(br)
                if cval < 0:
                    return None
            for _ in range(self.cdim[c]):
                book = self.subbooks[c][cval & ((1 << cbits) - 1)]
                cval >>= cbits
                if book >= 0:
                    e = books[book].decode(br)
                    if e < 0:
                        return None
                    Y.append(e)
                else:
                    Y.append(0)
        if br.eop:
            return None
        fy, step2 = self.final_y(Y)
        return self.curve(fy, step2, n2)


def bark(x):
    return 13.1 * math.atan(.00074 * x) + 2.24 * math.atan(.0000000185 * x * x) + .0001 * x


class Floor0:
    def __init__(self, br, nbooks):
        self.order, self.rate, self.bark_size = br.get(8), br.get(16), br.get(16)
        self.amp_bits, self.amp_offset = br.get(6), br.get(8)
        self.books = [br.get(8) for _ in range(br.get(4) + 1)]

    def curve(self, amp, coef, n2):  # Vorbis I 6.2.3 (f64)
        bn = bark(0.5 * self.rate)
        mp = [min(self.bark_size - 1, int(math.floor(bark(self.rate * i / (2.0 * n2)) * self.bark_size / bn)))
              for i in range(n2)] + [-1]
        cc = [math.cos(float(c)) for c in coef]
        out = np.zeros(n2, np.float32)
        i = 0
        while i < n2:
            cw = math.cos(math.pi * mp[i] / self.bark_size)
            if self.order & 1:
                p = 1.0 - cw * cw
                for j in range((self.order - 3) // 2 + 1):
                    p *= 4.0 * (cc[2 * j + 1] - cw) ** 2
                q = 0.25
                for j in range((self.order - 1) // 2 + 1):
                    q *= 4.0 * (cc[2 * j] - cw) ** 2
            else:
                p = (1.0 - cw) / 2.0
                for j in range((self.order - 2) // 2 + 1):
                    p *= 4.0 * (cc[2 * j + 1] - cw) ** 2
                q = (1.0 + cw) / 2.0
                for j in range((self.order - 2) // 2 + 1):
                    q *= 4.0 * (cc[2 * j] - cw) ** 2
            lin = math.exp(0.11512925 * (amp * self.amp_offset / ((1 << self.amp_bits) - 1) / math.sqrt(p + q)
                                         - self.amp_offset))
            m = mp[i]
            while i < n2 and mp[i] == m:
                out[i] = np.float32(lin)
                i += 1
        return out

    def decode(self, br, books, n2):
        amp = br.get(self.amp_bits)
        if br.eop or amp == 0:
            return None
        bn = br.get(ilog(len(self.books)))
        if br.eop or bn >= len(self.books):
            return None
        cb = books[self.books[bn]]
        coef, last = [], np.float32(0)
        while len(coef) < self.order:
            e = cb.decode(br)
            if e < 0:
                return None
            for v in cb.vq[e]:
                coef.append(np.float32(v + last))
            last = coef[-1]
        return self.curve(amp, coef, n2)


class Residue:
    def __init__(self, br, books):
        self.type = br.get(16)
        if self.type > 2:
            raise ValueError("Vorbis: bad residue type")
        self.begin, self.end, self.psize = br.get(24), br.get(24), br.get(24) + 1
        self.classes, self.classbook = br.get(6) + 1, br.get(8)
        casc = []
        for _ in range(self.classes):
            low = br.get(3)
            high = br.get(5) if br.get(1) else 0
            casc.append(high * 8 + low)
        self.books = [[br.get(8) if c & (1 << p) else -1 for p in range(8)] for c in casc]

    def decode01(self, br, books, fmt, vecs, dnd, n):
        """Formats 0 / 1 (Vorbis I 8.6.2-4), in place on vecs."""
        lb, le = min(self.begin, n), min(self.end, n)
        if le - lb <= 0:
            return
        nparts = (le - lb) // self.psize
        cbk = books[self.classbook]
        cpw = cbk.dims
        cls = [[0] * (nparts + cpw) for _ in vecs]
        for pas in range(8):
            pc = 0
            while pc < nparts:
                if pas == 0:
                    for j in range(len(vecs)):
                        if dnd[j]:
                            continue
                        temp = cbk.decode(br)
                        if temp < 0:
                            return
                        for i in range(cpw - 1, -1, -1):
                            cls[j][i + pc] = temp % self.classes
                            temp //= self.classes
                i = 0
                while i < cpw and pc < nparts:
                    for j in range(len(vecs)):
                        if dnd[j]:
                            continue
                        bk = self.books[cls[j][pc]][pas]
                        if bk < 0:
                            continue
                        cb = books[bk]
                        o = lb + pc * self.psize
                        if fmt == 0:
                            step = self.psize // cb.dims
                            for s in range(step):
                                e = cb.decode(br)
                                if e < 0:
                                    return
                                for k in range(cb.dims):
                                    vecs[j][o + s + k * step] += cb.vq[e, k]
                        else:
                            s = 0
                            while s < self.psize:
                                e = cb.decode(br)
                                if e < 0:
                                    return
                                for k in range(cb.dims):
                                    if s >= self.psize:
                                        break
                                    vecs[j][o + s] += cb.vq[e, k]
                                    s += 1
                    i += 1
                    pc += 1


_IMDCT = {}


def imdct(X):
    """y[n] = sum_k X[k] cos(2 pi/N (n + 1/2 + N/4)(k + 1/2)), N = 2 len(X) (f64 matrix)."""
    N = 2 * len(X)
    if N not in _IMDCT:
        n = np.arange(N)[:, None]
        k = np.arange(N // 2)[None, :]
        _IMDCT[N] = np.cos(2 * np.pi / N * (n + 0.5 + N / 4) * (k + 0.5))
    return (_IMDCT[N] @ X.astype(np.float64)).astype(np.float32)


def window(n, bs0, long_block, prev_long, next_long):  # Vorbis I 4.3.1
    w = np.zeros(n, np.float32)
    if long_block and not prev_long:
        ls, le, ln = n // 4 - bs0 // 4, n // 4 + bs0 // 4, bs0 // 2
    else:
        ls, le, ln = 0, n // 2, n // 2
    if long_block and not next_long:
        rs, re, rn = n * 3 // 4 - bs0 // 4, n * 3 // 4 + bs0 // 4, bs0 // 2
    else:
        rs, re, rn = n // 2, n, n // 2
    for i in range(ls, le):
        s = math.sin((i - ls + 0.5) / ln * math.pi / 2)
        w[i] = math.sin(math.pi / 2 * s * s)
    w[le:rs] = 1.0
    for i in range(rs, re):
        s = math.sin((i - rs + 0.5) / rn * math.pi / 2 + math.pi / 2)
        w[i] = math.sin(math.pi / 2 * s * s)
    return w


class Decoder:
    def __init__(self, ident: bytes, setup: bytes):
        if ident[:7] != b"\x01vorbis":
            raise ValueError("Vorbis: bad identification header")
        br = Bits(ident[7:])
        if br.get(32) != 0:
            raise ValueError("Vorbis: version")
        self.channels, self.rate = br.get(8), br.get(32)
        br.get(32), br.get(32), br.get(32)
        self.bs = (1 << br.get(4), 1 << br.get(4))
        if not br.get(1):
            raise ValueError("Vorbis: framing")
        if setup[:7] != b"\x05vorbis":
            raise ValueError("Vorbis: bad setup header")
        br = Bits(setup[7:])
        self.books = [Codebook(br) for _ in range(br.get(8) + 1)]
        for _ in range(br.get(6) + 1):
            if br.get(16) != 0:
                raise ValueError("Vorbis: time domain transform")
        self.floors = []
        for _ in range(br.get(6) + 1):
            t = br.get(16)
            self.floors.append(Floor0(br, len(self.books)) if t == 0 else Floor1(br, len(self.books)))
        self.residues = [Residue(br, self.books) for _ in range(br.get(6) + 1)]
        self.maps = []
        for _ in range(br.get(6) + 1):
            if br.get(16) != 0:
                raise ValueError("Vorbis: mapping type")
            sub = br.get(4) + 1 if br.get(1) else 1
            mag, ang = [], []
            if br.get(1):
                for _ in range(br.get(8) + 1):
                    mag.append(br.get(ilog(self.channels - 1)))
                    ang.append(br.get(ilog(self.channels - 1)))
            if br.get(2):
                raise ValueError("Vorbis: mapping reserved")
            mux = [br.get(4) for _ in range(self.channels)] if sub > 1 else [0] * self.channels
            sf, sr = [], []
            for _ in range(sub):
                br.get(8)
                sf.append(br.get(8))
                sr.append(br.get(8))
            self.maps.append(dict(sub=sub, mag=mag, ang=ang, mux=mux, floor=sf, res=sr))
        self.modes = []
        for _ in range(br.get(6) + 1):
            bf = br.get(1)
            br.get(16), br.get(16)
            self.modes.append((bf, br.get(8)))
        if not br.get(1):
            raise ValueError("Vorbis: setup framing")

    def audio(self, pkt: bytes):
        """One audio packet -> (n, windowed block [channels, n], nonzero span) or None."""
        br = Bits(pkt)
        if not pkt or br.get(1) != 0:
            return None
        mn = br.get(ilog(len(self.modes) - 1))
        if br.eop or mn >= len(self.modes):
            return None
        bf, mi = self.modes[mn]
        n = self.bs[bf]
        n2 = n // 2
        pl = nl = 1
        if bf:
            pl, nl = br.get(1), br.get(1)
        m = self.maps[mi]
        C = self.channels
        floors = [self.floors[m["floor"][m["mux"][c]]].decode(br, self.books, n2) for c in range(C)]
        no_res = [f is None for f in floors]
        for a, b in zip(m["mag"], m["ang"]):
            if not no_res[a] or not no_res[b]:
                no_res[a] = no_res[b] = False
        res = [np.zeros(n2, np.float32) for _ in range(C)]
        for s in range(m["sub"]):
            chs = [c for c in range(C) if m["mux"][c] == s]
            r = self.residues[m["res"][s]]
            dnd = [no_res[c] for c in chs]
            if r.type == 2:
                if all(dnd):
                    continue
                tmp = [np.zeros(n2 * len(chs), np.float32)]
                r.decode01(br, self.books, 1, tmp, [False], n2 * len(chs))
                for i, c in enumerate(chs):
                    res[c] = tmp[0][i::len(chs)].copy()
            else:
                vecs = [res[c] for c in chs]
                r.decode01(br, self.books, r.type, vecs, dnd, n2)
        for a, b in reversed(list(zip(m["mag"], m["ang"]))):  # inverse coupling (4.3.5)
            M, A = res[a], res[b]
            for j in range(n2):
                m0, a0 = M[j], A[j]
                if m0 > 0:
                    nm, na = (m0, m0 - a0) if a0 > 0 else (m0 + a0, m0)
                else:
                    nm, na = (m0, m0 + a0) if a0 > 0 else (m0 - a0, m0)
                M[j], A[j] = nm, na
        w = window(n, self.bs[0], bf, pl, nl)
        blk = np.zeros((C, n), np.float32)
        for c in range(C):
            if floors[c] is None:
                continue
            blk[c] = imdct((res[c] * floors[c]).astype(np.float32)) * w
        ls = n // 4 - self.bs[0] // 4 if (bf and not pl) else 0
        re = n * 3 // 4 + self.bs[0] // 4 if (bf and not nl) else n
        return n, blk, ls, re


def decode(data: bytes):
    """Ogg Vorbis bytes -> (float32 [frames, channels], sample_rate)."""
    pk, last_page = read_packets(data)
    if len(pk) < 3 or pk[1][0][:7] != b"\x03vorbis":
        raise ValueError("Vorbis: missing headers")
    D = Decoder(pk[0][0], pk[2][0])
    C = D.channels
    acc = np.zeros((C, 0), np.float32)
    p, prev_n, prev_c, first_c, produced = D.bs[1], 0, None, None, 0
    start_trim, end_total, seen = 0, None, False
    for data_, gran, page in pk[3:]:
        r = D.audio(data_)
        if r is not None:
            n, blk, ls, re = r
            if prev_n:
                p += 3 * prev_n // 4 - n // 4
            if acc.shape[1] < p + n:
                acc = np.concatenate([acc, np.zeros((C, p + n - acc.shape[1]), np.float32)], axis=1)
            acc[:, p + ls:p + re] += blk[:, ls:re]
            center = p + n // 2
            if prev_c is None:
                first_c = center
            else:
                produced += center - prev_c
            prev_c, prev_n = center, n
        if gran >= 0:
            last = page == last_page
            if not seen and not last and gran < produced:
                start_trim = produced - gran
            seen = True
            if last:
                end_total = gran
    total = produced - start_trim
    if end_total is not None:
        total = min(total, end_total)
    total = max(total, 0)
    if first_c is None:
        return np.zeros((0, C), np.float32), D.rate
    s0 = first_c + start_trim
    return np.ascontiguousarray(acc[:, s0:s0 + total].T), D.rate
