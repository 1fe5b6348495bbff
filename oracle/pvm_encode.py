"""PVM / DDS writer for the reader's tests.  TEST INFRASTRUCTURE ONLY.

Restates the V^3 Differential Data Stream encoder that libs/file_utils/pvm.cpp
carries commented out (:681-841, DDS_encode; :914-975, writePVMvolume): the
bytes are de-interleaved with stride `skip`, each byte is predicted from the
previous one (and, past the first `strip` bytes, from the difference of the two
bytes one `strip` earlier), and the prediction errors are written in runs of
up to 127 with a per-run bit width (codes 0..7 -> widths 0, 2..8), MSB-first in
big-endian 32-bit words.  Runs here are cut greedily by width (the reference's
encoder merges runs by a cost model; any grouping is a valid stream for the
decoder).  The reference repository ships no .pvm file, so these streams are
what pins cvr_read_pvm: round trips of volumes through this writer.
"""
from __future__ import annotations

import numpy as np


class _Bits:
    def __init__(self):
        self.words = []
        self.buf = 0
        self.n = 0

    def write(self, value: int, bits: int):
        for k in range(bits - 1, -1, -1):
            self.buf = (self.buf << 1) | ((value >> k) & 1)
            self.n += 1
            if self.n == 32:
                self.words.append(self.buf)
                self.buf, self.n = 0, 0

    def bytes(self) -> bytes:
        out = b"".join(w.to_bytes(4, "big") for w in self.words)
        if self.n:
            tail = (self.buf << (32 - self.n)).to_bytes(4, "big")
            out += tail[: (self.n + 7) // 8]          # DDS_flushbits: whole bytes only
        return out


def _width(delta: int) -> int:
    """Smallest representable width whose biased range holds delta (lookup[] + code)."""
    if delta <= 0:
        b = 0
        while (1 << b) // 2 < -delta:
            b += 1
    else:
        b = 0
        while (1 << b) // 2 <= delta:
            b += 1
    return 2 if b == 1 else b          # DDS_decode(DDS_code(1)) = 2


def dds_encode(data: bytes, skip: int = 1, strip: int = 1) -> bytes:
    d = np.frombuffer(data, np.uint8)
    n = d.size
    if skip > 1:                        # DDS_deinterleave(restore = false), block 0
        d = np.concatenate([d[i::skip] for i in range(skip)])
    d = d.astype(np.int64)
    deltas = []
    pre = 0
    for i in range(n):
        t = int(d[i])
        if strip == 1 or i <= strip:
            a = t - pre
        else:
            a = t - pre - int(d[i - strip]) + int(d[i - strip - 1])
        pre = t
        while a < -128:
            a += 256
        while a > 127:
            a -= 256
        deltas.append(a)
    bw = _Bits()
    bw.write(skip - 1, 2)
    bw.write(strip - 1, 16)
    i = 0
    while i < n:
        b = _width(deltas[i])
        j = i + 1
        while j < n and j - i < 127 and _width(deltas[j]) <= b:
            j += 1
        bw.write(j - i, 7)
        bw.write(b - 1 if b > 1 else b, 3)             # DDS_code
        for k in range(i, j):
            bw.write(deltas[k] + (1 << b) // 2, b)
        i = j
    bw.write(0, 7)                                      # end of stream
    return bw.bytes()


def pvm_payload(vol: np.ndarray, version: int = 2, scale=(1.0, 1.0, 1.0),
                strings=("", "", "", "")) -> bytes:
    """writePVMvolume's payload: header + voxels (+ 4 strings for PVM3).  u16 volumes
    are stored low byte first, the order the reference's reader assembles."""
    d, h, w = vol.shape
    comps = vol.dtype.itemsize
    if version == 1:
        head = f"PVM\n{w} {h} {d}\n{comps}\n"
    else:
        head = f"PVM{version}\n{w} {h} {d}\n{scale[0]:g} {scale[1]:g} {scale[2]:g}\n{comps}\n"
    body = vol.astype("<u2" if comps == 2 else np.uint8).tobytes()
    tail = b""
    if version == 3:
        tail = b"".join(s.encode() + b"\0" for s in strings)
    return head.encode() + body + tail


def write_pvm(path: str, vol: np.ndarray, version: int = 2, scale=(1.0, 1.0, 1.0),
              compress: bool = True, skip: int = 1, strip: int = 1, v3e: bool = False,
              strings=("", "", "", "")):
    payload = pvm_payload(vol, version, scale, strings)
    with open(path, "wb") as f:
        if compress:
            f.write(b"DDS v3e\n" if v3e else b"DDS v3d\n")
            f.write(dds_encode(payload, skip, strip))
        else:
            f.write(payload)
