"""``NetworkBuffer`` — the reference's only serialised layout, byte-compatible
(NetworkBuffer.cs:29-847; layout comment :32-45, commands :109-126, parser
``oku`` :137-194, header write ``buf`` :600-614).

Layout (little-endian)::

    "Cekirdek"            8 bytes magic
    endianness            1 byte (0 = little endian)
    total length          int32 (bytes, whole buffer)  @ offset 9
    command               int32                          @ offset 13
    records ...           from offset 17

    record = type u8 | hash i32 | length i32 | [ref i32 | range i32]  (float only)
             | payload (length elements, or `range` elements for a partial
             float record: elements [ref, ref+range) of the array)

A partial float record carries element units on the wire, as the reference
writes them (``addArray(float[])`` multiplies the work-item offset and range
by elements-per-work-item, NetworkBuffer.cs:764-790, and ``oku`` advances
``menzil·4`` bytes, :182): ``add_array(a, h, ref, range_, epw)`` takes work
items and writes ``ref·epw`` / ``range_·epw``, and :meth:`NetworkBuffer.parse`
needs nothing out of band.

Element types: 0=byte 1=char(16-bit) 2=int32 3=float32 4=int64 5=float64
6=bool.  This layout is used for the cluster wire protocol
(:mod:`cekirdekler_amd.parallel.cluster`) and for checkpoints
(:mod:`cekirdekler_amd.utils.checkpoint`).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

MAGIC = b"Cekirdek"
HEADER = 17

# commands (NetworkBuffer.cs:109-126)
SETUP = 0
COMPUTE = 1
DISPOSE = 2
ANSWER_SUCCESS = 3
ANSWER_DELETED = 4
ANSWER_COMPUTE_COMPLETE = 5
SERVER_STOP = 6
ANSWER_STOPPED = 7
SERVER_CONTROL = 8
ANSWER_CONTROL = 9
SERVER_NUMBER_OF_DEVICES = 10
ANSWER_NUMBER_OF_DEVICES = 11
# extensions of this framework (values past the reference's range)
CHECKPOINT = 64
ANSWER_ERROR = 65

TYPE_BYTE, TYPE_CHAR, TYPE_INT, TYPE_FLOAT, TYPE_LONG, TYPE_DOUBLE, TYPE_BOOL = range(7)
_TYPE_DTYPE = {TYPE_BYTE: np.uint8, TYPE_CHAR: np.uint16, TYPE_INT: np.int32, TYPE_FLOAT: np.float32,
               TYPE_LONG: np.int64, TYPE_DOUBLE: np.float64, TYPE_BOOL: np.bool_}
_DTYPE_TYPE = {np.dtype(np.uint8): TYPE_BYTE, np.dtype(np.int8): TYPE_BYTE,
               np.dtype(np.uint16): TYPE_CHAR, np.dtype(np.int16): TYPE_CHAR,
               np.dtype(np.int32): TYPE_INT, np.dtype(np.uint32): TYPE_INT,
               np.dtype(np.float32): TYPE_FLOAT, np.dtype(np.int64): TYPE_LONG,
               np.dtype(np.uint64): TYPE_LONG, np.dtype(np.float64): TYPE_DOUBLE,
               np.dtype(np.bool_): TYPE_BOOL}


def type_code(dtype) -> int:
    dt = np.dtype(dtype)
    if dt not in _DTYPE_TYPE:
        raise TypeError(f"NetworkBuffer cannot carry dtype {dt}")
    return _DTYPE_TYPE[dt]


@dataclass
class Record:
    type: int
    hash: int
    length: int          # elements of the whole array
    ref: int = 0         # partial float records: first element
    range: int = -1      # partial float records: elements carried (-1 = all)
    data: Optional[np.ndarray] = None

    def scatter_into(self, a: np.ndarray) -> None:
        """Writes the record's payload into ``a`` where the sender took it
        from (element offset ``ref``; the whole array for a full record)."""
        if self.partial:
            if self.range > 0:
                a[self.ref:self.ref + self.range] = self.data
        elif len(self.data) == len(a):
            a[:] = self.data

    @property
    def partial(self) -> bool:
        return self.type == TYPE_FLOAT and self.range != -1


class NetworkBuffer:
    """Builder/parser for the reference wire format."""

    def __init__(self, command: int = -1):
        self.command = command
        self._parts: List[bytes] = []
        self._size = HEADER

    # ------------------------------------------------------------- building
    def add_array(self, arr: np.ndarray, hash_: int, ref: int = 0, range_: int = -1, epw: int = 1) -> None:
        a = np.ascontiguousarray(arr).reshape(-1)
        t = type_code(a.dtype)
        if t == TYPE_BOOL:
            a = a.astype(np.uint8)
        head = struct.pack("<Bii", t, _i32(hash_), len(a))
        if t == TYPE_FLOAT:
            lo, n = (int(ref) * epw, int(range_) * epw) if range_ != -1 else (0, -1)
            head += struct.pack("<ii", lo, n)
            payload = a[lo:lo + n] if n != -1 else a
        else:
            if range_ != -1:
                raise ValueError("partial records exist only for float arrays (reference layout)")
            payload = a
        self._parts.append(head)
        self._parts.append(payload.view(np.uint8).tobytes())
        self._size += len(head) + payload.nbytes

    def add_string(self, s: str, hash_: int = 0) -> None:
        self.add_array(np.frombuffer(s.encode("utf-16-le"), dtype=np.uint16), hash_)

    def add_ints(self, values, hash_: int = 0) -> None:
        self.add_array(np.asarray(values, dtype=np.int32), hash_)

    def add_doubles(self, values, hash_: int = 0) -> None:
        self.add_array(np.asarray(values, dtype=np.float64), hash_)

    def to_bytes(self) -> bytes:
        head = MAGIC + bytes([0]) + struct.pack("<ii", self._size, int(self.command))
        return head + b"".join(self._parts)

    buf = to_bytes

    def __len__(self) -> int:
        return self._size

    # ------------------------------------------------------------- parsing
    @staticmethod
    def read_length(b: bytes) -> int:
        if b[:8] != MAGIC:
            raise ValueError("not a Cekirdekler NetworkBuffer")
        return struct.unpack_from("<i" if b[8] == 0 else ">i", b, 9)[0]

    @staticmethod
    def parse(b: bytes):
        """Returns (command, [Record])."""
        if b[:8] != MAGIC:
            raise ValueError("not a Cekirdekler NetworkBuffer")
        e = "<" if b[8] == 0 else ">"
        total, command = struct.unpack_from(e + "ii", b, 9)
        mv = memoryview(b)
        i = HEADER
        out: List[Record] = []
        while i < total:
            t = b[i]
            h, n = struct.unpack_from(e + "ii", b, i + 1)
            i += 9
            ref, rng = 0, -1
            if t == TYPE_FLOAT:
                ref, rng = struct.unpack_from(e + "ii", b, i)
                i += 8
            dt = np.dtype(_TYPE_DTYPE[t] if t != TYPE_BOOL else np.uint8).newbyteorder(e)
            count = n if rng == -1 else rng
            data = np.frombuffer(mv[i:i + count * dt.itemsize], dtype=dt)
            if t == TYPE_BOOL:
                data = data.astype(np.bool_)
            out.append(Record(t, h, n, ref, rng, data))
            i += count * dt.itemsize
        return command, out

    @staticmethod
    def record_string(r: Record) -> str:
        return r.data.astype("<u2").tobytes().decode("utf-16-le")

    # ---- the reference's spellings (NetworkBuffer.cs:52-830) ----------------
    SETUP, COMPUTE, DISPOSE = SETUP, COMPUTE, DISPOSE
    ANSWER_SUCCESS, ANSWER_DELETED, ANSWER_COMPUTE_COMPLETE = ANSWER_SUCCESS, ANSWER_DELETED, ANSWER_COMPUTE_COMPLETE
    SERVER_STOP, ANSWER_STOPPED, SERVER_CONTROL, ANSWER_CONTROL = (SERVER_STOP, ANSWER_STOPPED, SERVER_CONTROL,
                                                                  ANSWER_CONTROL)
    SERVER_NUMBER_OF_DEVICES, ANSWER_NUMBER_OF_DEVICES = SERVER_NUMBER_OF_DEVICES, ANSWER_NUMBER_OF_DEVICES
    receiveSendBufferSize = 8 * 1024  # socket send/receive buffer (NetworkBuffer.cs:52)

    def bufferCommand(self) -> int:  # noqa: N802
        return int(self.command)

    def komutBelirle(self, k: int) -> None:  # noqa: N802  (set the command)
        self.command = int(k)

    @staticmethod
    def komutOku(b: bytes) -> int:  # noqa: N802  (read the command of a serialized buffer)
        return NetworkBuffer.parse(b)[0]

    readLengthOfBuffer = read_length

    def elemanSay(self) -> int:  # noqa: N802  (number of records)
        return len(self._parts) // 2

    def addArray(self, arr, hash_: int, ref: int = 0, range_: int = -1, epw: int = 1) -> None:  # noqa: N802
        self.add_array(np.asarray(arr), hash_, ref, range_, epw)

    @staticmethod
    def oku(b: bytes):
        """Parse a serialized buffer: (command, records) (NetworkBuffer.oku)."""
        return NetworkBuffer.parse(b)


def _i32(v: int) -> int:
    v = int(v) & 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v
