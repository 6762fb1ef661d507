"""Test-only FLAC encoder (RFC 9639) that produces every bitstream feature the
decoder in libaa.so (csrc/aa_flac.cpp) must handle: CONSTANT, VERBATIM, FIXED
0-4 and LPC subframes, wasted bits, partitioned Rice residuals with 4- and
5-bit parameters and escape partitions, the three stereo decorrelations,
fixed and variable block-size streams, every header code for block size,
sample rate and bit depth, and unknown stream length.  No FLAC encoder or
decoder is installed in the image (ffmpeg, libFLAC and soundfile are absent),
so decode parity is against this restatement of the specification and the
catalogue check values of its CRCs -- parity unpinned against ffmpeg.
"""
from __future__ import annotations

import numpy as np


def crc8(data: bytes) -> int:  # CRC-8, poly x^8 + x^2 + x + 1, init 0
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data: bytes) -> int:  # CRC-16, poly x^16 + x^15 + x^2 + 1, init 0
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


class Bits:
    def __init__(self):
        self.parts = []
        self.n = 0

    def put(self, v: int, k: int):
        if k:
            self.parts.append(format(v & ((1 << k) - 1), f"0{k}b"))
            self.n += k

    def raw(self, s: str):
        self.parts.append(s)
        self.n += len(s)

    def tobytes(self) -> bytes:
        s = "".join(self.parts)
        s += "0" * (-len(s) % 8)
        return int(s, 2).to_bytes(len(s) // 8, "big") if s else b""


def _utf8(v: int) -> bytes:
    if v < 0x80:
        return bytes([v])
    for n in range(2, 8):
        if v < (1 << (5 * n + 1)) or n == 7:
            out = []
            for _ in range(n - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            lead = (0xFF << (8 - n)) & 0xFF
            return bytes([lead | v] + out[::-1])
    raise ValueError(v)


_FIXED = {0: [], 1: [1], 2: [2, -1], 3: [3, -3, 1], 4: [4, -6, 4, -1]}


def _rice_partition(bits: Bits, u: np.ndarray, k: int):
    mask = (1 << k) - 1
    for x in u.tolist():
        bits.raw("0" * (x >> k) + "1" + (format(x & mask, f"0{k}b") if k else ""))


def _residual(bits: Bits, res: np.ndarray, block: int, order: int, porder: int, method: int, escape_parts=()):
    bits.put(method, 2)
    bits.put(porder, 4)
    pbits, esc = (4, 15) if method == 0 else (5, 31)
    per = block >> porder
    i = 0
    for p in range(1 << porder):
        cnt = per - (order if p == 0 else 0)
        r = res[i:i + cnt]
        i += cnt
        if p in escape_parts:
            nb = 0 if not len(r) or not np.any(r) else int(max(abs(int(r.min())), int(r.max()))).bit_length() + 1
            bits.put(esc, pbits)
            bits.put(nb, 5)
            for x in r.tolist():
                bits.put(x, nb)
            continue
        u = np.where(r >= 0, 2 * r, -2 * r - 1).astype(np.int64) if len(r) else r.astype(np.int64)
        mean = float(u.mean()) if len(u) else 0.0
        k = max(0, int(np.log2(mean)) if mean >= 1 else 0)
        k = min(k, esc - 1)
        bits.put(k, pbits)
        _rice_partition(bits, u, k)


def _lpc_coefs(s: np.ndarray, order: int, prec: int):
    """least-squares predictor quantised to `prec` signed bits with a shift"""
    x = s.astype(np.float64)
    if len(x) <= order * 2:
        a = np.zeros(order)
    else:
        A = np.stack([x[order - 1 - j: len(x) - 1 - j] for j in range(order)], axis=1)
        a = np.linalg.lstsq(A, x[order:], rcond=None)[0]
    cmax = np.max(np.abs(a)) if np.any(a) else 1.0
    shift = max(0, min(15, prec - 1 - int(np.ceil(np.log2(cmax + 1e-12))) - 1))
    q = np.clip(np.round(a * (1 << shift)), -(1 << (prec - 1)), (1 << (prec - 1)) - 1).astype(np.int64)
    return q, shift


def _predict(s: np.ndarray, coefs, shift: int) -> np.ndarray:
    order = len(coefs)
    res = s.astype(np.int64).copy()
    for i in range(order, len(s)):
        acc = 0
        for j, c in enumerate(coefs):
            acc += int(c) * int(s[i - 1 - j])
        res[i] = int(s[i]) - (acc >> shift)
    return res[order:]


def subframe(bits: Bits, s: np.ndarray, bps: int, kind: str, order: int = 0, wasted: int = 0,
             porder: int = 0, method: int = 0, escape_parts=(), prec: int = 12):
    """kind: constant | verbatim | fixed | lpc; s already within bps bits"""
    block = len(s)
    if wasted:
        assert np.all((s & ((1 << wasted) - 1)) == 0)
        s = s >> wasted
        bps -= wasted
    code = {"constant": 0, "verbatim": 1}.get(kind)
    if kind == "fixed":
        code = 8 + order
    elif kind == "lpc":
        code = 31 + order
    bits.put(0, 1)
    bits.put(code, 6)
    if wasted:
        bits.put(1, 1)
        bits.raw("0" * (wasted - 1) + "1")
    else:
        bits.put(0, 1)
    if kind == "constant":
        assert np.all(s == s[0])
        bits.put(int(s[0]), bps)
        return
    if kind == "verbatim":
        for x in s.tolist():
            bits.put(x, bps)
        return
    for x in s[:order].tolist():
        bits.put(x, bps)
    if kind == "fixed":
        res = _predict(s, _FIXED[order], 0)
    else:
        coefs, shift = _lpc_coefs(s, order, prec)
        bits.put(prec - 1, 4)
        bits.put(shift, 5)
        for c in coefs.tolist():
            bits.put(c, prec)
        res = _predict(s, coefs, shift)
    _residual(bits, res, block, order, porder, method, escape_parts)


_BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12,
             8192: 13, 16384: 14, 32768: 15}
_SR_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
             48000: 10, 96000: 11}
_BPS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def frame(chans, bps: int, sr: int, number: int, stereo: str = "indep", kinds=None, sr_mode="table",
          bps_mode="table", bs_mode="table", variable=False) -> bytes:
    """One frame of int64 channel arrays (equal length).  kinds: per channel a
    dict of subframe() keyword arguments."""
    block = len(chans[0])
    nch = len(chans)
    hdr = Bits()
    hdr.put(0x3FFE, 14)
    hdr.put(0, 1)
    hdr.put(1 if variable else 0, 1)
    bs_code = _BS_CODES.get(block) if bs_mode == "table" else None
    if bs_code is None:
        bs_code = 6 if block <= 256 and bs_mode != "16" else 7
    if sr_mode == "table" and sr in _SR_CODES:
        sr_code = _SR_CODES[sr]
    elif sr_mode == "khz":
        sr_code = 12
    elif sr_mode == "dahz":
        sr_code = 14
    elif sr_mode == "streaminfo":
        sr_code = 0
    else:
        sr_code = 13
    hdr.put(bs_code, 4)
    hdr.put(sr_code, 4)
    ch_code = {"indep": nch - 1, "left_side": 8, "side_right": 9, "mid_side": 10}[stereo]
    hdr.put(ch_code, 4)
    hdr.put(_BPS_CODES[bps] if bps_mode == "table" and bps in _BPS_CODES else 0, 3)
    hdr.put(0, 1)
    head = hdr.tobytes() + _utf8(number)
    if bs_code == 6:
        head += bytes([block - 1])
    elif bs_code == 7:
        head += (block - 1).to_bytes(2, "big")
    if sr_code == 12:
        head += bytes([sr // 1000])
    elif sr_code == 13:
        head += sr.to_bytes(2, "big")
    elif sr_code == 14:
        head += (sr // 10).to_bytes(2, "big")
    head += bytes([crc8(head)])
    body = Bits()
    c = [np.asarray(x, np.int64) for x in chans]
    if stereo == "left_side":
        coded, extra = [c[0], c[0] - c[1]], [0, 1]
    elif stereo == "side_right":
        coded, extra = [c[0] - c[1], c[1]], [1, 0]
    elif stereo == "mid_side":
        coded, extra = [(c[0] + c[1]) >> 1, c[0] - c[1]], [0, 1]
    else:
        coded, extra = c, [0] * nch
    kinds = kinds or [{"kind": "fixed", "order": 2}] * nch
    for x, e, kw in zip(coded, extra, kinds):
        subframe(body, x, bps + e, **kw)
    data = head + body.tobytes()
    return data + crc16(data).to_bytes(2, "big")


def stream(frames_bytes, sr: int, channels: int, bps: int, total: int, max_block: int,
           extra_blocks=(), id3: bytes = b"") -> bytes:
    si = Bits()
    si.put(16 if max_block >= 16 else max_block, 16)
    si.put(max_block, 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(sr, 20)
    si.put(channels - 1, 3)
    si.put(bps - 1, 5)
    si.put(total, 36)
    si.put(0, 128)
    blocks = [(0, si.tobytes())] + list(extra_blocks)
    out = bytearray(id3 + b"fLaC")
    for i, (t, body) in enumerate(blocks):
        out.append((0x80 if i == len(blocks) - 1 else 0) | t)
        out += len(body).to_bytes(3, "big")
        out += body
    for f in frames_bytes:
        out += f
    return bytes(out)
