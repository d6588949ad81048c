"""TEST INFRASTRUCTURE: a small FLAC encoder written from the format specification (RFC 9639), used only
to make fixtures for the native decoder (taiwan-whisper_amd/csrc/flac.cpp, tw_flac_decode).  It emits
every construct the decoder reads: STREAMINFO (with the MD5 of the samples), frame headers with each
block-size / sample-rate / sample-size coding (and CRC-8), CONSTANT / VERBATIM / FIXED (orders 0-4) /
LPC subframes, wasted bits, Rice partitions of any order with 4- or 5-bit parameters and escaped
(raw) partitions, independent / left-side / side-right / mid-side stereo, CRC-16 footers.
No libFLAC / soundfile exists in this image, so the round trip (decode(encode(x)) == x bit for bit)
and the decoder's own CRC / MD5 checks are the parity test; a frame the RFC's published example file
holds is checked separately (tests/test_flac_cpu.py)."""
from __future__ import annotations

import hashlib

import numpy as np


class BitWriter:
    def __init__(self):
        self.buf = bytearray()
        self.acc = 0
        self.nbits = 0

    def write(self, v: int, k: int):
        if k == 0:
            return
        v &= (1 << k) - 1
        self.acc = (self.acc << k) | v
        self.nbits += k
        while self.nbits >= 8:
            self.nbits -= 8
            self.buf.append((self.acc >> self.nbits) & 0xFF)
        self.acc &= (1 << self.nbits) - 1

    def write_signed(self, v: int, k: int):
        self.write(v & ((1 << k) - 1), k)

    def unary(self, q: int):
        for _ in range(q // 32):
            self.write(0, 32)
        self.write(1, q % 32 + 1)

    def align(self):
        if self.nbits:
            self.write(0, 8 - self.nbits)

    def bytes(self) -> bytes:
        assert self.nbits == 0
        return bytes(self.buf)


def crc8(d: bytes) -> int:
    c = 0
    for x in d:
        c ^= x
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(d: bytes) -> int:
    c = 0
    for x in d:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _utf8_number(n: int) -> bytes:
    if n < 0x80:
        return bytes([n])
    for nb, lim in ((2, 1 << 11), (3, 1 << 16), (4, 1 << 21), (5, 1 << 26), (6, 1 << 31), (7, 1 << 36)):
        if n < lim:
            out = []
            for _ in range(nb - 1):
                out.append(0x80 | (n & 0x3F))
                n >>= 6
            lead = (0xFF << (8 - nb)) & 0xFF
            out.append(lead | n)
            return bytes(reversed(out))
    raise ValueError(n)


def _rice_cost(u: np.ndarray, k: int) -> int:
    return int(np.sum(u >> k)) + len(u) * (k + 1)


def _residual(bw: BitWriter, res: np.ndarray, bs: int, order: int, porder: int, escape_part: int | None,
              method: int = 0):
    """Rice-code res (the bs - order residuals) in 2^porder partitions."""
    bw.write(method, 2)
    bw.write(porder, 4)
    pbits, esc = (4, 15) if method == 0 else (5, 31)
    parts = 1 << porder
    per = bs >> porder
    i = 0
    for pt in range(parts):
        cnt = per - (order if pt == 0 else 0)
        r = res[i:i + cnt].astype(np.int64)
        i += cnt
        u = np.where(r >= 0, 2 * r, -2 * r - 1).astype(np.uint64) if cnt else np.zeros(0, np.uint64)
        if escape_part == pt:
            raw = int(max([int(abs(x)).bit_length() + 1 for x in r] + [1]))
            bw.write(esc, pbits)
            bw.write(raw, 5)
            for x in r:
                bw.write_signed(int(x), raw)
            continue
        k = min(range(esc), key=lambda kk: _rice_cost(u, kk)) if cnt else 0
        bw.write(k, pbits)
        for x in u:
            x = int(x)
            bw.unary(x >> k)
            bw.write(x & ((1 << k) - 1), k)


FIXED_COEF = {0: [], 1: [1], 2: [2, -1], 3: [3, -3, 1], 4: [4, -6, 4, -1]}


def _subframe(bw: BitWriter, s: np.ndarray, bps: int, kind: str, porder: int = 0, escape_part=None,
              lpc_order: int = 8, lpc_prec: int = 12, wasted: bool = True, method: int = 0):
    s = s.astype(np.int64)
    bs = len(s)
    w = 0
    if wasted and np.any(s != 0):
        while np.all((s >> (w + 1) << (w + 1)) == s) and w + 1 < bps:
            w += 1
    bw.write(0, 1)
    if kind == "constant":
        assert np.all(s == s[0])
        bw.write(0, 6)
    elif kind == "verbatim":
        bw.write(1, 6)
    elif kind.startswith("fixed"):
        bw.write(8 + int(kind[5:]), 6)
    elif kind == "lpc":
        bw.write(31 + lpc_order, 6)
    if w:
        bw.write(1, 1)
        bw.unary(w - 1)
    else:
        bw.write(0, 1)
    x = s >> w
    bb = bps - w
    if kind == "constant":
        bw.write_signed(int(x[0]), bb)
    elif kind == "verbatim":
        for v in x:
            bw.write_signed(int(v), bb)
    elif kind.startswith("fixed"):
        order = int(kind[5:])
        for v in x[:order]:
            bw.write_signed(int(v), bb)
        c = FIXED_COEF[order]
        pred = np.zeros(bs, np.int64)
        for j, cj in enumerate(c):
            pred[order:] += cj * x[order - 1 - j: bs - 1 - j]
        _residual(bw, (x - pred)[order:], bs, order, porder, escape_part, method)
    else:
        order = lpc_order
        for v in x[:order]:
            bw.write_signed(int(v), bb)
        # least-squares predictor, quantised to lpc_prec bits with the largest shift that fits
        X = np.stack([x[order - 1 - j: bs - 1 - j] for j in range(order)], 1).astype(np.float64)
        coef = np.linalg.lstsq(X, x[order:].astype(np.float64), rcond=None)[0] if bs > 2 * order else np.zeros(order)
        cmax = max(np.abs(coef).max(), 1e-9)
        shift = max(0, min(15, lpc_prec - 1 - int(np.ceil(np.log2(cmax + 1e-12))) - 1))
        q = np.clip(np.round(coef * (1 << shift)), -(1 << (lpc_prec - 1)), (1 << (lpc_prec - 1)) - 1).astype(np.int64)
        bw.write(lpc_prec - 1, 4)
        bw.write_signed(shift, 5)
        for cq in q:
            bw.write_signed(int(cq), lpc_prec)
        pred = np.zeros(bs, np.int64)
        for i in range(order, bs):
            pred[i] = int(np.dot(q, x[i - 1::-1][:order])) >> shift
        _residual(bw, (x - pred)[order:], bs, order, porder, escape_part, method)


BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12, 8192: 13,
            16384: 14, 32768: 15}
SR_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9, 48000: 10,
            96000: 11}
SS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def encode(samples: np.ndarray, sample_rate: int = 16000, bps: int = 16, block_size: int = 4096,
           stereo: str = "independent", kinds=("fixed2",), porder: int = 0, escape_part=None,
           header_rate_code: str = "table", header_bs_code: str = "table", wasted: bool = True,
           method: int = 0, id3: bool = False) -> bytes:
    """samples: int array [n] or [n, ch].  kinds: subframe kind per frame (cycled); stereo: independent |
    left_side | side_right | mid_side (2 channels).  header_*_code: 'table' uses the standard code when
    there is one, 'explicit' the 8/16-bit in-header forms, 'streaminfo' code 0."""
    x = np.asarray(samples, np.int64)
    if x.ndim == 1:
        x = x[:, None]
    n, ch = x.shape
    out = bytearray()
    if id3:
        out += b"ID3\x03\x00\x00\x00\x00\x00\x05" + b"\x00" * 5
    out += b"fLaC"
    si = BitWriter()
    si.write(block_size, 16)
    si.write(block_size, 16)
    si.write(0, 24)
    si.write(0, 24)
    si.write(sample_rate, 20)
    si.write(ch - 1, 3)
    si.write(bps - 1, 5)
    si.write(n, 36)
    nbytes = (bps + 7) // 8
    inter = x.reshape(-1)
    raw = b"".join(int(v).to_bytes(nbytes, "little", signed=True) for v in inter)
    md5 = hashlib.md5(raw).digest()
    siv = si.bytes() + md5
    out += bytes([0x80, 0, 0, len(siv)]) + siv            # last metadata block: STREAMINFO
    fi = 0
    for a in range(0, n, block_size):
        blk = x[a:a + block_size]
        bs = len(blk)
        hb = BitWriter()
        hb.write(0x3FFE, 14)
        hb.write(0, 1)
        hb.write(0, 1)                                   # fixed blocking
        tail = BitWriter()
        if header_bs_code == "table" and bs in BS_CODES:
            hb.write(BS_CODES[bs], 4)
        elif bs <= 256:
            hb.write(6, 4)
            tail.write(bs - 1, 8)
        else:
            hb.write(7, 4)
            tail.write(bs - 1, 16)
        if header_rate_code == "streaminfo":
            hb.write(0, 4)
        elif header_rate_code == "table" and sample_rate in SR_CODES:
            hb.write(SR_CODES[sample_rate], 4)
        elif sample_rate % 1000 == 0 and sample_rate // 1000 < 256 and header_rate_code != "hz":
            hb.write(12, 4)
            tail.write(sample_rate // 1000, 8)
        elif sample_rate < 65536:
            hb.write(13, 4)
            tail.write(sample_rate, 16)
        else:
            hb.write(14, 4)
            tail.write(sample_rate // 10, 16)
        if ch == 2 and stereo != "independent":
            hb.write({"left_side": 8, "side_right": 9, "mid_side": 10}[stereo], 4)
        else:
            hb.write(ch - 1, 4)
        hb.write(SS_CODES[bps] if header_rate_code != "streaminfo" else 0, 3)
        hb.write(0, 1)
        head = hb.bytes() + _utf8_number(fi) + tail.bytes()
        head += bytes([crc8(head)])
        body = BitWriter()
        chans = [blk[:, c] for c in range(ch)]
        cb = [bps] * ch
        if ch == 2 and stereo == "left_side":
            chans, cb = [blk[:, 0], blk[:, 0] - blk[:, 1]], [bps, bps + 1]
        elif ch == 2 and stereo == "side_right":
            chans, cb = [blk[:, 0] - blk[:, 1], blk[:, 1]], [bps + 1, bps]
        elif ch == 2 and stereo == "mid_side":
            chans, cb = [(blk[:, 0] + blk[:, 1]) >> 1, blk[:, 0] - blk[:, 1]], [bps, bps + 1]
        kind = kinds[fi % len(kinds)]
        for c in range(ch):
            k = kind
            if k == "constant" and not np.all(chans[c] == chans[c][0]):
                k = "verbatim"
            if (k.startswith("fixed") and int(k[5:]) > bs) or (k == "lpc" and bs <= 16):
                k = "verbatim"
            po = porder
            while po and ((bs >> po) < 32 or bs % (1 << po)):
                po -= 1
            ep = escape_part if escape_part is None or escape_part < (1 << po) else None
            _subframe(body, chans[c], cb[c], k, po, ep, wasted=wasted, method=method)
        body.align()
        frame = head + body.bytes()
        frame += crc16(frame).to_bytes(2, "big")
        out += frame
        fi += 1
    return bytes(out)
