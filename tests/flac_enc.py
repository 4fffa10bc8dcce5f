"""A FLAC encoder for the tests (test infrastructure, never used by the product).

Writes every bitstream feature amx_flac_decode reads (RFC 9639): STREAMINFO plus other
metadata blocks, fixed- and variable-blocksize frame headers with every block-size and
sample-rate code form, CONSTANT / VERBATIM / FIXED (orders 0-4) / LPC subframes, wasted
bits, Rice partitions with 4- and 5-bit parameters and escapes, the four channel
assignments, CRC-8 and CRC-16.  The decoder is pinned by the round trip: decode(encode(x))
must give x back bit for bit for every combination.
"""
import numpy as np


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, k):
        """k low bits of v (k <= 64)"""
        if k == 0:
            return
        self.acc = (self.acc << k) | (int(v) & ((1 << k) - 1))
        self.n += k
        while self.n >= 8:
            self.n -= 8
            self.out.append((self.acc >> self.n) & 0xFF)
        self.acc &= (1 << self.n) - 1

    def sput(self, v, k):
        self.put(int(v) & ((1 << k) - 1), k)

    def unary(self, q):
        while q >= 32:
            self.put(0, 32)
            q -= 32
        self.put(1, q + 1)

    def align(self):
        if self.n:
            self.put(0, 8 - self.n)

    def bytes(self):
        assert self.n == 0
        return bytes(self.out)


def crc8(b):
    c = 0
    for x in b:
        c ^= x
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(b):
    c = 0
    for x in b:
        c ^= x << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


def _utf8(v):
    if v < 0x80:
        return bytes([v])
    for nb in range(2, 8):
        if v < (1 << (5 * nb + 1)) or nb == 7:
            out = []
            for _ in range(nb - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            lead = (0xFF << (8 - nb)) & 0xFF if nb < 7 else 0xFE
            out.append(lead | v)
            return bytes(reversed(out))
    raise ValueError(v)


BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12,
            8192: 13, 16384: 14, 32768: 15}
SR_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8,
            44100: 9, 48000: 10, 96000: 11}
SS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def _rice_residual(w, res, rng, order, block):
    """partitioned Rice residual: a random partition order the block allows, parameters
    from the partition's mean, 5-bit parameters when needed, an escape now and then"""
    res = [int(v) for v in res]
    po = 0
    cands = [p for p in range(0, 5) if block % (1 << p) == 0 and (block >> p) >= order]
    po = int(rng.choice(cands))
    big = max([abs(v) for v in res] + [0]) >= (1 << 13)
    method = 1 if big or rng.random() < 0.3 else 0
    w.put(method, 2)
    w.put(po, 4)
    pbits = 5 if method else 4
    esc = (1 << pbits) - 1
    n = block >> po
    i = 0
    for p in range(1 << po):
        cnt = n - (order if p == 0 else 0)
        part = res[i:i + cnt]
        i += cnt
        u = [((v << 1) ^ -1) if v < 0 else (v << 1) for v in part]
        mean = (sum(u) / len(u)) if u else 0
        k = max(0, int(np.log2(mean + 1))) if mean > 0 else 0
        if k >= esc or rng.random() < 0.08:
            nb = max([abs(v).bit_length() + 1 for v in part] + [1]) if part else 0
            nb = min(max(nb, 0), 31)
            w.put(esc, pbits)
            w.put(nb, 5)
            for v in part:
                w.sput(v, nb) if nb else None
        else:
            w.put(k, pbits)
            for v in u:
                w.unary(v >> k)
                w.put(v & ((1 << k) - 1), k)


def _subframe(w, x, bps, rng, kind):
    """one channel's samples x (ints of bps bits) as the subframe kind"""
    x = [int(v) for v in x]
    block = len(x)
    wasted = 0
    if rng.random() < 0.3 and any(x):
        t = min((v & -v).bit_length() - 1 for v in x if v)
        wasted = min(t, bps - 1)
    xs = [v >> wasted for v in x]
    eb = bps - wasted
    if kind == "constant" and len(set(xs)) == 1:
        w.put(0, 1)
        w.put(0, 6)
        _wasted(w, wasted)
        w.sput(xs[0], eb)
        return
    if kind == "verbatim":
        w.put(0, 1)
        w.put(1, 6)
        _wasted(w, wasted)
        for v in xs:
            w.sput(v, eb)
        return
    if kind.startswith("fixed"):
        order = min(int(kind[5:]), block)
        w.put(0, 1)
        w.put(8 + order, 6)
        _wasted(w, wasted)
        for v in xs[:order]:
            w.sput(v, eb)
        res = []
        for i in range(order, block):
            s = xs
            pred = [0, s[i - 1], 2 * s[i - 1] - s[i - 2] if i >= 2 else 0,
                    3 * s[i - 1] - 3 * s[i - 2] + s[i - 3] if i >= 3 else 0,
                    4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4] if i >= 4 else 0][order]
            res.append(s[i] - pred)
        _rice_residual(w, res, rng, order, block)
        return
    # LPC: random order 1..12, precision and shift, coefficients near a smoothing predictor
    order = min(int(rng.integers(1, 13)), block)
    prec = int(rng.integers(4, 16))
    shift = int(rng.integers(0, min(prec, 15) + 1))
    lim = 1 << (prec - 1)
    coef = [int(np.clip(round((2.0 if k == 0 else (-1.0 if k == 1 else 0.0)) * (1 << shift) * rng.uniform(0.5, 1.0)),
                        -lim, lim - 1)) for k in range(order)]
    w.put(0, 1)
    w.put(31 + order, 6)
    _wasted(w, wasted)
    for v in xs[:order]:
        w.sput(v, eb)
    w.put(prec - 1, 4)
    w.sput(shift, 5)
    for c in coef:
        w.sput(c, prec)
    res = []
    for i in range(order, block):
        acc = sum(coef[k] * xs[i - 1 - k] for k in range(order))
        res.append(xs[i] - (acc >> shift))
    _rice_residual(w, res, rng, order, block)


def _wasted(w, wasted):
    if wasted:
        w.put(1, 1)
        w.unary(wasted - 1)
    else:
        w.put(0, 1)


def encode(x, fs, bps, seed=0, block=4096, variable=False, kinds=None, assigns=None, metadata=True,
           stream_bps_in_header=None):
    """FLAC bytes of x (int array [frames, channels] of bps-bit signed samples)."""
    rng = np.random.default_rng(seed)
    x = np.asarray(x, np.int64)
    if x.ndim == 1:
        x = x[:, None]
    n, ch = x.shape
    kinds = kinds or ["verbatim", "fixed0", "fixed1", "fixed2", "fixed3", "fixed4", "lpc", "constant"]
    assigns = assigns or ([0, 8, 9, 10] if ch == 2 else [0])
    frames = []
    pos = 0
    fno = 0
    sizes = []
    while pos < n:
        b = block if not variable else int(rng.integers(16, 2 * block))
        b = min(b, n - pos)
        seg = x[pos:pos + b]
        w = BitWriter()
        w.put(0x3FFE, 14)
        w.put(0, 1)
        w.put(1 if variable else 0, 1)
        if b in BS_CODES and rng.random() < 0.7:
            bsc, bsx = BS_CODES[b], None
        elif b <= 256:
            bsc, bsx = 6, (b - 1, 8)
        else:
            bsc, bsx = 7, (b - 1, 16)
        r = rng.random()
        if r < 0.4:
            src, srx = 0, None
        elif fs in SR_CODES and r < 0.7:
            src, srx = SR_CODES[fs], None
        elif fs % 10 == 0 and fs // 10 < 65536 and r < 0.85:
            src, srx = 14, (fs // 10, 16)
        elif fs < 65536:
            src, srx = 13, (fs, 16)
        else:
            src, srx = 0, None
        a = int(rng.choice(assigns)) if ch == 2 else ch - 1
        if a < 8:
            a = ch - 1                                    # independent channels: code = channels - 1
        w.put(bsc, 4)
        w.put(src, 4)
        w.put(a, 4)
        ssc = 0 if rng.random() < 0.5 or bps not in SS_CODES else SS_CODES[bps]
        w.put(ssc, 3)
        w.put(0, 1)
        for byte in _utf8(pos if variable else fno):
            w.put(byte, 8)
        if bsx:
            w.put(*bsx)
        if srx:
            w.put(*srx)
        hdr = w.bytes()
        w.put(crc8(hdr), 8)
        chans = [seg[:, c] for c in range(ch)]
        side_bps = [bps] * ch
        if ch == 2 and a >= 8:
            l, rr = seg[:, 0], seg[:, 1]
            side = l - rr
            if a == 8:
                chans, side_bps = [l, side], [bps, bps + 1]
            elif a == 9:
                chans, side_bps = [side, rr], [bps + 1, bps]
            else:
                chans, side_bps = [(l + rr) >> 1, side], [bps, bps + 1]
        for c in range(ch):
            k = str(rng.choice(kinds))
            _subframe(w, chans[c], side_bps[c], rng, k)
        w.align()
        body = w.bytes()
        frame = body + crc16(body).to_bytes(2, "big")
        frames.append(frame)
        sizes.append(b)
        pos += b
        fno += 1
    # metadata: STREAMINFO (+ PADDING and an APPLICATION block)
    si = BitWriter()
    si.put(min(sizes) if len(sizes) > 1 else sizes[0], 16)
    si.put(max(sizes), 16)
    si.put(min(len(f) for f in frames), 24)
    si.put(max(len(f) for f in frames), 24)
    si.put(fs, 20)
    si.put(ch - 1, 3)
    si.put(bps - 1, 5)
    si.put(n, 36)
    si.put(0, 128)
    blocks = [(0, si.bytes())]
    if metadata:
        blocks += [(2, b"test" + bytes(12)), (1, bytes(37))]
    out = bytearray(b"fLaC")
    for i, (t, body) in enumerate(blocks):
        last = 1 if i == len(blocks) - 1 else 0
        out.append((last << 7) | t)
        out += len(body).to_bytes(3, "big")
        out += body
    for f in frames:
        out += f
    return bytes(out)
