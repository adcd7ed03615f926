"""Determinant types and the host-side encoder (DeterminantEncoder.encode mirror).

Encoding stays on the host (in Clonos it is Java: SimpleDeterminantEncoder.encodeTo,
reference flink-runtime/.../causal/determinant/SimpleDeterminantEncoder.java:56-75 and
the per-type writers :124-323).  This module restates the byte layout so the Python host
mirror, the tests and the synthetic workload generators can produce records; decoding is
done on the GPU (Engine.decode_*).

Byte layouts (big-endian, tag first):
  ORDER             [00][channel i8]                                        2 B
  TIMESTAMP         [01][ts i64]                                            9 B
  RNG               [02][number i32]                                        5 B
  SERIALIZABLE      [03][java serialization stream]                         1 + len
  TIMER_TRIGGER     [04][recordCount i32][ts i64][type u8]{[len i32][name]} 14 / 18 + len
  SOURCE_CHECKPOINT [05][rc i32][cp i64][ts i64][type u8][hasRef u8]{[len i32][ref]} 23 / 27 + len
  IGNORE_CHECKPOINT [06][rc i32][cp i64]                                    13 B
  BUFFER_BUILT      [07][bytes i32]                                         5 B
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Optional, Union

ORDER, TIMESTAMP, RNG, SERIALIZABLE, TIMER_TRIGGER, SOURCE_CHECKPOINT, IGNORE_CHECKPOINT, BUFFER_BUILT = range(8)
TAG_NAMES = ["ORDER", "TIMESTAMP", "RNG", "SERIALIZABLE", "TIMER_TRIGGER", "SOURCE_CHECKPOINT",
             "IGNORE_CHECKPOINT", "BUFFER_BUILT"]
WIDE_TAGS = (SERIALIZABLE, TIMER_TRIGGER, SOURCE_CHECKPOINT, IGNORE_CHECKPOINT)

# ProcessingTimeCallbackID.Type (ProcessingTimeCallbackID.java:33-34)
WATERMARK, TIMESTAMP_EXTRACTOR, TIMESTAMP_PERIODIC_WATERMARK_EXTRACTOR, \
    TIMESTAMP_PUNCTUATED_WATERMARK_EXTRACTOR, IDLE, LATENCY, INTERNAL = range(7)
# CheckpointType (checkpoint/CheckpointType.java:27,30)
CHECKPOINT, SAVEPOINT = 0, 1


@dataclass
class OrderDeterminant:
    channel: int  # Java byte


@dataclass
class TimestampDeterminant:
    timestamp: int


@dataclass
class RNGDeterminant:
    number: int


@dataclass
class BufferBuiltDeterminant:
    number_of_bytes: int


@dataclass
class SerializableDeterminant:
    stream: bytes  # one complete ObjectOutputStream stream (AC ED 00 05 ...)


@dataclass
class TimerTriggerDeterminant:
    record_count: int
    timestamp: int
    callback_type: int = INTERNAL
    name: Optional[bytes] = None  # only for INTERNAL


@dataclass
class SourceCheckpointDeterminant:
    record_count: int
    checkpoint_id: int
    checkpoint_timestamp: int
    checkpoint_type: int = CHECKPOINT
    storage_reference: Optional[bytes] = field(default=b"")


@dataclass
class IgnoreCheckpointDeterminant:
    record_count: int
    checkpoint_id: int


Determinant = Union[OrderDeterminant, TimestampDeterminant, RNGDeterminant, BufferBuiltDeterminant,
                    SerializableDeterminant, TimerTriggerDeterminant, SourceCheckpointDeterminant,
                    IgnoreCheckpointDeterminant]


def _i8(v: int) -> int:
    return ((v + 128) & 0xFF) - 128


def _i32(v: int) -> int:
    return ((v + (1 << 31)) & 0xFFFFFFFF) - (1 << 31)


def _i64(v: int) -> int:
    return ((v + (1 << 63)) & 0xFFFFFFFFFFFFFFFF) - (1 << 63)


def encode(d: Determinant) -> bytes:
    """SimpleDeterminantEncoder.encode (:35-53)."""
    if isinstance(d, OrderDeterminant):
        return struct.pack(">Bb", ORDER, _i8(d.channel))
    if isinstance(d, TimestampDeterminant):
        return struct.pack(">Bq", TIMESTAMP, _i64(d.timestamp))
    if isinstance(d, RNGDeterminant):
        return struct.pack(">Bi", RNG, _i32(d.number))
    if isinstance(d, BufferBuiltDeterminant):
        return struct.pack(">Bi", BUFFER_BUILT, _i32(d.number_of_bytes))
    if isinstance(d, SerializableDeterminant):
        return bytes([SERIALIZABLE]) + bytes(d.stream)
    if isinstance(d, TimerTriggerDeterminant):
        out = struct.pack(">BiqB", TIMER_TRIGGER, _i32(d.record_count), _i64(d.timestamp), d.callback_type & 0xFF)
        if d.callback_type == INTERNAL:
            name = d.name or b""
            out += struct.pack(">i", len(name)) + name
        return out
    if isinstance(d, SourceCheckpointDeterminant):
        ref = d.storage_reference
        out = struct.pack(">BiqqBB", SOURCE_CHECKPOINT, _i32(d.record_count), _i64(d.checkpoint_id),
                          _i64(d.checkpoint_timestamp), d.checkpoint_type & 0xFF, 0 if ref is None else 1)
        if ref is not None:
            out += struct.pack(">i", len(ref)) + ref
        return out
    if isinstance(d, IgnoreCheckpointDeterminant):
        return struct.pack(">Biq", IGNORE_CHECKPOINT, _i32(d.record_count), _i64(d.checkpoint_id))
    raise TypeError(f"UnknownDeterminantTypeException: {type(d).__name__}")


def encoded_size(d: Determinant) -> int:
    """Determinant.getEncodedSizeInBytes (the per-class overrides)."""
    return len(encode(d))


def timer_name(name: str) -> bytes:
    """String.getBytes() of a timer name; ASCII in practice ("PTS", "87", ...)."""
    return name.encode("utf-8")


# ---- Java Object Serialization writer (subset) ---------------------------------------
# Streams exactly as java.io.ObjectOutputStream writes them for a fresh stream holding
# one object (Java Object Serialization Specification, section 6).  Used to build
# SERIALIZABLE determinants (SerializableCausalService.apply writes the user object).
_MAGIC = b"\xac\xed\x00\x05"


def _utf(s: str) -> bytes:
    b = s.encode("utf-8")
    return struct.pack(">H", len(b)) + b


def jser_string(s: str) -> bytes:
    return _MAGIC + b"\x74" + _utf(s)


def jser_null() -> bytes:
    return _MAGIC + b"\x70"


def jser_boolean(v: bool) -> bytes:
    return (_MAGIC + b"\x73\x72" + _utf("java.lang.Boolean") + bytes.fromhex("cd207280d59cfaee") + b"\x02"
            + b"\x00\x01" + b"Z" + _utf("value") + b"\x78\x70" + (b"\x01" if v else b"\x00"))


def _number_desc() -> bytes:
    return b"\x72" + _utf("java.lang.Number") + bytes.fromhex("86ac951d0b94e08b") + b"\x02\x00\x00\x78\x70"


def jser_integer(v: int) -> bytes:
    return (_MAGIC + b"\x73\x72" + _utf("java.lang.Integer") + bytes.fromhex("12e2a0a4f7818738") + b"\x02"
            + b"\x00\x01" + b"I" + _utf("value") + b"\x78" + _number_desc() + struct.pack(">i", _i32(v)))


def jser_long(v: int) -> bytes:
    return (_MAGIC + b"\x73\x72" + _utf("java.lang.Long") + bytes.fromhex("3b8be490cc8f23df") + b"\x02"
            + b"\x00\x01" + b"J" + _utf("value") + b"\x78" + _number_desc() + struct.pack(">q", _i64(v)))


def jser_int_array(vals) -> bytes:
    return (_MAGIC + b"\x75\x72" + _utf("[I") + bytes.fromhex("4dba602676eab2a5") + b"\x02\x00\x00\x78\x70"
            + struct.pack(">i", len(vals)) + b"".join(struct.pack(">i", _i32(v)) for v in vals))
