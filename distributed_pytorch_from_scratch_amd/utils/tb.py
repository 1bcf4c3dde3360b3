"""Minimal TensorBoard event-file writer (scalars), no tensorboard/tensorboardX dependency.

Reference parity: the reference logs with ``tensorboardX.SummaryWriter`` (``train.py:85,117-120``,
``test.py:112,121``); neither tensorboard nor tensorboardX is installed on the MI355X image,
so this writes the same on-disk format directly: a TFRecord stream of ``Event`` protobufs
(``events.out.tfevents.<ts>.<host>``), each record = len(u64) | masked-crc32c(len) | data |
masked-crc32c(data).  TensorBoard reads these files as-is.  ``SummaryWriter`` exposes the
subset the reference uses: ``add_scalar(tag, value, step)``, ``flush()``, ``close()``.
"""
from __future__ import annotations

import os
import socket
import struct
import time

_CRC_TABLE = None


def _crc32c(data: bytes) -> int:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        poly = 0x82F63B78
        tab = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            tab.append(c)
        _CRC_TABLE = tab
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def _masked(crc: int) -> int:
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field(num: int, wire: int, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _event(wall_time: float, step: int, *, file_version: str = None, tag: str = None, value: float = None) -> bytes:
    msg = _field(1, 1, struct.pack("<d", wall_time)) + _field(2, 0, _varint(step))
    if file_version is not None:
        fv = file_version.encode()
        msg += _field(3, 2, _varint(len(fv)) + fv)
    if tag is not None:
        t = tag.encode()
        val = _field(1, 2, _varint(len(t)) + t) + _field(2, 5, struct.pack("<f", float(value)))
        summary = _field(1, 2, _varint(len(val)) + val)
        msg += _field(5, 2, _varint(len(summary)) + summary)
    return msg


class SummaryWriter:
    def __init__(self, log_dir: str):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self._f = open(self.path, "ab")
        self._write(_event(time.time(), 0, file_version="brain.Event:2"))

    def _write(self, data: bytes):
        header = struct.pack("<Q", len(data))
        self._f.write(header + struct.pack("<I", _masked(_crc32c(header))) + data
                      + struct.pack("<I", _masked(_crc32c(data))))

    def add_scalar(self, tag: str, value: float, global_step: int = 0):
        self._write(_event(time.time(), int(global_step), tag=tag, value=float(value)))

    def flush(self):
        self._f.flush()

    def close(self):
        if not self._f.closed:
            self._f.flush()
            self._f.close()


def read_scalars(path: str):
    """Parse an event file written by ``SummaryWriter`` -> list of (step, tag, value)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i + 12 <= len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        rec = data[i + 12:i + 12 + n]
        i += 12 + n + 4
        step, tag, val, j = 0, None, None, 0

        def rd_varint(buf, k):
            v, s = 0, 0
            while True:
                b = buf[k]
                k += 1
                v |= (b & 0x7F) << s
                s += 7
                if not b & 0x80:
                    return v, k

        while j < len(rec):
            key, j = rd_varint(rec, j)
            num, wire = key >> 3, key & 7
            if wire == 0:
                v, j = rd_varint(rec, j)
                if num == 2:
                    step = v
            elif wire == 1:
                j += 8
            elif wire == 5:
                j += 4
            elif wire == 2:
                ln, j = rd_varint(rec, j)
                payload = rec[j:j + ln]
                j += ln
                if num == 5:  # summary -> value -> (tag, simple_value)
                    k = 0
                    _, k = rd_varint(payload, k)
                    vl, k = rd_varint(payload, k)
                    vb = payload[k:k + vl]
                    m = 0
                    while m < len(vb):
                        kk, m = rd_varint(vb, m)
                        if kk >> 3 == 1:
                            tl, m = rd_varint(vb, m)
                            tag = vb[m:m + tl].decode()
                            m += tl
                        elif kk >> 3 == 2:
                            val = struct.unpack_from("<f", vb, m)[0]
                            m += 4
        if tag is not None:
            out.append((step, tag, val))
    return out
