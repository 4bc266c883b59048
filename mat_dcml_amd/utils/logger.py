"""Self-contained scalar logger with the reference's ``SummaryWriter`` surface.

The reference logs through tensorboardX ``add_scalars`` (``base_runner.py:60-63``; ``dcml_runner.py:110-117,317``)
and exports ``logs/summary.json`` at the end (``DCML_MAT_Train.py:182``); tensorboard/tensorboardX are not
installed here, so this writer keeps the same calls and tag names and writes:

* ``logs/scalars.jsonl`` — one JSON object per scalar (tag, step, wall time, value);
* ``logs/<tag>.csv`` — ``Wall time,Step,Value`` like the published TensorBoard CSV exports
  (``data/dcml_benchmark/momat_ct.csv``);
* ``logs/events.out.tfevents.*`` — a minimal TF-event file (hand-encoded protobuf + masked CRC32C) that
  TensorBoard can read when it is available elsewhere;
* ``export_scalars_to_json`` → ``summary.json`` ({tag: [[wall, step, value], ...]}).

The reference writes delay AND payment to the same tag ``train_episode_scores/aver_scores`` (the second
overwrites the first, §2.7 #6); here they are ``train_episode_scores/aver_delay`` and ``.../aver_payment``.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time


def _crc32c_table():
    tbl = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        tbl.append(c)
    return tbl


_TBL = _crc32c_table()


def _crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TBL[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def _masked_crc(data: bytes) -> int:
    c = _crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


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


def _field(num, wire, payload: bytes) -> bytes:
    return _varint((num << 3) | wire) + payload


def _event_bytes(wall, step, tag=None, value=None, file_version=None) -> bytes:
    ev = _field(1, 1, struct.pack("<d", wall)) + _field(2, 0, _varint(int(step)))
    if file_version is not None:
        fv = file_version.encode()
        ev += _field(3, 2, _varint(len(fv)) + fv)
    if tag is not None:
        t = tag.encode()
        val = _field(1, 2, _varint(len(t)) + t) + _field(2, 5, struct.pack("<f", float(value)))
        summ = _field(1, 2, _varint(len(val)) + val)
        ev += _field(5, 2, _varint(len(summ)) + summ)
    return ev


class ScalarWriter:
    def __init__(self, log_dir: str, enabled: bool = True, tfevents: bool = True):
        self.log_dir = str(log_dir)
        self.enabled = enabled
        self.scalars = {}
        self._jsonl = None
        self._tf = None
        if enabled:
            os.makedirs(self.log_dir, exist_ok=True)
            self._jsonl = open(os.path.join(self.log_dir, "scalars.jsonl"), "a")
            if tfevents:
                fn = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
                self._tf = open(os.path.join(self.log_dir, fn), "ab")
                self._write_tf(_event_bytes(time.time(), 0, file_version="brain.Event:2"))

    def _write_tf(self, data: bytes):
        hdr = struct.pack("<Q", len(data))
        self._tf.write(hdr + struct.pack("<I", _masked_crc(hdr)) + data + struct.pack("<I", _masked_crc(data)))

    def add_scalar(self, tag, value, step):
        value = float(value)
        wall = time.time()
        self.scalars.setdefault(tag, []).append([wall, int(step), value])
        if not self.enabled or self._jsonl is None:   # disabled rank, or written after close()
            return
        self._jsonl.write(json.dumps({"tag": tag, "step": int(step), "wall": wall, "value": value}) + "\n")
        self._jsonl.flush()
        fn = os.path.join(self.log_dir, tag.replace("/", "_") + ".csv")
        new = not os.path.exists(fn)
        with open(fn, "a") as f:
            if new:
                f.write("Wall time,Step,Value\n")
            f.write(f"{wall},{int(step)},{value}\n")
        if self._tf is not None:
            self._write_tf(_event_bytes(wall, step, tag, value))
            self._tf.flush()

    def add_scalars(self, main_tag, tag_scalar_dict, step):
        for k, v in tag_scalar_dict.items():
            self.add_scalar(f"{main_tag}/{k}", v, step)

    def export_scalars_to_json(self, path):
        if self.enabled:
            with open(path, "w") as f:
                json.dump(self.scalars, f)

    def close(self):
        for fh in (self._jsonl, self._tf):
            if fh is not None:
                fh.close()
        self._jsonl = self._tf = None
