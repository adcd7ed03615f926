"""Seeded synthetic determinant logs for the BASELINE.json configurations.

Vectorised with numpy: every record *kind* has a fixed length and a byte template;
per-record fields (channel, timestamp, counts, ...) are patched big-endian into the
template copies.  Record layouts follow SimpleDeterminantEncoder (see determinants.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import determinants as D

SEED_CONFIG2 = 0xC1050002
SEED_CONFIG3 = 0xC1050003


@dataclass
class Kind:
    name: str
    template: bytes
    patches: Tuple[Tuple[int, int], ...]  # (position, width) of big-endian fields
    wide: bool


def _kinds() -> Dict[str, Kind]:
    k = {}
    k["order"] = Kind("order", D.encode(D.OrderDeterminant(0)), ((1, 1),), False)
    k["timestamp"] = Kind("timestamp", D.encode(D.TimestampDeterminant(0)), ((1, 8),), False)
    k["rng"] = Kind("rng", D.encode(D.RNGDeterminant(0)), ((1, 4),), False)
    k["buffer_built"] = Kind("buffer_built", D.encode(D.BufferBuiltDeterminant(0)), ((1, 4),), False)
    # "PTS": StreamTask time-setter timer (StreamTask.java:1519) -> 21 B
    k["timer_pts"] = Kind("timer_pts", D.encode(D.TimerTriggerDeterminant(0, 0, D.INTERNAL, b"PTS")),
                          ((1, 4), (5, 8)), True)
    # window timer "W".hashCode() % 1000 = "87" (WindowOperator.java:203) -> 20 B
    k["timer_87"] = Kind("timer_87", D.encode(D.TimerTriggerDeterminant(0, 0, D.INTERNAL, b"87")),
                         ((1, 4), (5, 8)), True)
    k["source_cp"] = Kind("source_cp", D.encode(D.SourceCheckpointDeterminant(0, 0, 0, D.CHECKPOINT, b"")),
                          ((1, 4), (5, 8), (13, 8)), True)
    k["ignore_cp"] = Kind("ignore_cp", D.encode(D.IgnoreCheckpointDeterminant(0, 0)), ((1, 4), (5, 8)), True)
    k["ser_string"] = Kind("ser_string", D.encode(D.SerializableDeterminant(D.jser_string("abc"))), (), True)
    sb = D.encode(D.SerializableDeterminant(D.jser_boolean(True)))
    k["ser_boolean"] = Kind("ser_boolean", sb, ((len(sb) - 1, 1),), True)
    si = D.encode(D.SerializableDeterminant(D.jser_integer(0)))
    k["ser_integer"] = Kind("ser_integer", si, ((len(si) - 4, 4),), True)
    return k


KINDS = _kinds()


def _be_bytes(vals: np.ndarray, width: int) -> np.ndarray:
    v = vals.astype(np.uint64)
    shifts = np.arange(width - 1, -1, -1, dtype=np.uint64) * np.uint64(8)
    return ((v[:, None] >> shifts[None, :]) & np.uint64(0xFF)).astype(np.uint8)


def build(kind_idx: np.ndarray, kinds: Sequence[Kind], fields: Dict[int, List[np.ndarray]]) -> Tuple[np.ndarray, np.ndarray]:
    """Lay out records: kind_idx[i] selects kinds[k]; fields[k][j] holds patch j's values for
    the records of kind k (in order).  Returns (bytes, record offsets)."""
    lens = np.array([len(k.template) for k in kinds], np.int64)[kind_idx]
    offs = np.zeros(len(kind_idx) + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    buf = np.empty(int(offs[-1]), np.uint8)
    for ki, kd in enumerate(kinds):
        sel = np.nonzero(kind_idx == ki)[0]
        if sel.size == 0:
            continue
        t = np.frombuffer(kd.template, np.uint8)
        pos = offs[sel][:, None] + np.arange(len(t))[None, :]
        buf[pos] = t[None, :]
        for j, (p, w) in enumerate(kd.patches):
            vals = fields.get(ki, [None] * len(kd.patches))[j]
            if vals is None:
                continue
            buf[offs[sel][:, None] + p + np.arange(w)[None, :]] = _be_bytes(vals, w)
    return buf, offs[:-1]


def config2_log(n_records: int, rng: np.random.Generator, channels: int = 4) -> Tuple[np.ndarray, np.ndarray]:
    """Config 2: tag ~ Bernoulli(0.5) Order/Timestamp, channel ~ U[0, channels),
    timestamps from 1.7e12 ms with +U[0,5] increments."""
    kinds = [KINDS["order"], KINDS["timestamp"]]
    kind_idx = (rng.random(n_records) < 0.5).astype(np.int64)
    n_ts = int(kind_idx.sum())
    ch = rng.integers(0, channels, n_records - n_ts)
    ts = 1_700_000_000_000 + np.cumsum(rng.integers(0, 6, n_ts))
    return build(kind_idx, kinds, {0: [ch], 1: [ts]})


SEED_CONFIG4 = 0xC1050004


def config4_epoch(table, gids: np.ndarray, rng: np.random.Generator, main_records: int = 4096,
                  sub_records: int = 64) -> Tuple[np.ndarray, np.ndarray]:
    """Config 4 (5-stage DAG, p=128, full sharing): one epoch of every log in `gids`
    (job.LogTable indices), back to back.  Main-thread logs: `main_records` Order/Timestamp
    determinants (the config-2 mix); subpartition logs: `sub_records` BufferBuilt
    determinants (one per output buffer, PipelinedSubpartition.java:370).  Returns
    (bytes, per-log byte offsets with a final end offset)."""
    is_main = np.array([table.ids[int(g)].is_main for g in gids], bool)
    n_sub = int((~is_main).sum())
    kd = KINDS["buffer_built"]
    sub_blk, _ = build(np.zeros(n_sub * sub_records, np.int64), [kd],
                       {0: [rng.integers(1, 32769, n_sub * sub_records)]})
    sub_len = sub_records * len(kd.template)
    parts, k = [], 0
    for m in is_main:
        if m:
            parts.append(config2_log(main_records, rng)[0])
        else:
            parts.append(sub_blk[k * sub_len:(k + 1) * sub_len])
            k += 1
    offs = np.zeros(len(parts) + 1, np.uint64)
    np.cumsum([p.size for p in parts], out=offs[1:])
    return (np.concatenate(parts) if parts else np.zeros(0, np.uint8)), offs


CONFIG3_MIX = [("order", 0.35), ("buffer_built", 0.35), ("timer_pts", 0.05), ("timer_87", 0.05),
               ("timestamp", 0.05), ("rng", 0.05), ("ser_string", 0.05 / 3), ("ser_boolean", 0.05 / 3),
               ("ser_integer", 0.05 / 3), ("source_cp", 0.03), ("ignore_cp", 0.02)]


def config3_epoch(n_records: int, rng: np.random.Generator, epoch: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Config 3: mixed variable-length determinants incl. Serializable and BufferBuilt."""
    names = [n for n, _ in CONFIG3_MIX]
    p = np.array([w for _, w in CONFIG3_MIX])
    kinds = [KINDS[n] for n in names]
    kind_idx = rng.choice(len(kinds), size=n_records, p=p / p.sum())
    fields: Dict[int, List[np.ndarray]] = {}
    for ki, kd in enumerate(kinds):
        cnt = int((kind_idx == ki).sum())
        vals = []
        for (pos, w) in kd.patches:
            if kd.name == "order":
                vals.append(rng.integers(0, 4, cnt))
            elif kd.name in ("timestamp",) or (w == 8 and pos in (5, 13) and kd.name.startswith("timer")):
                vals.append(1_700_000_000_000 + rng.integers(0, 10_000, cnt))
            elif kd.name == "buffer_built":
                vals.append(rng.integers(1, 32768, cnt))
            elif w == 8:
                vals.append(np.full(cnt, epoch, np.int64) if pos == 5 else 1_700_000_000_000 + rng.integers(0, 10_000, cnt))
            elif kd.name == "ser_boolean":
                vals.append(rng.integers(0, 2, cnt))
            else:
                vals.append(rng.integers(0, 1 << 31, cnt))
        fields[ki] = vals
    return build(kind_idx, kinds, fields)


def random_determinant(rng: np.random.Generator, allow_serializable: bool = True) -> D.Determinant:
    """Arbitrary-valued determinant of any type (tests)."""
    t = int(rng.integers(0, 8 if allow_serializable else 7))
    if not allow_serializable and t >= 3:
        t += 1
    r = lambda lo, hi: int(rng.integers(lo, hi))  # noqa: E731
    if t == D.ORDER:
        return D.OrderDeterminant(r(-128, 128))
    if t == D.TIMESTAMP:
        return D.TimestampDeterminant(r(-(1 << 62), 1 << 62))
    if t == D.RNG:
        return D.RNGDeterminant(r(-(1 << 31), 1 << 31))
    if t == D.BUFFER_BUILT:
        return D.BufferBuiltDeterminant(r(0, 1 << 31))
    if t == D.SERIALIZABLE:
        c = r(0, 6)
        if c == 0:
            return D.SerializableDeterminant(D.jser_string("x" * r(0, 40)))
        if c == 1:
            return D.SerializableDeterminant(D.jser_boolean(bool(r(0, 2))))
        if c == 2:
            return D.SerializableDeterminant(D.jser_integer(r(-(1 << 31), 1 << 31)))
        if c == 3:
            return D.SerializableDeterminant(D.jser_long(r(-(1 << 62), 1 << 62)))
        if c == 4:
            return D.SerializableDeterminant(D.jser_int_array([r(0, 100) for _ in range(r(0, 30))]))
        return D.SerializableDeterminant(D.jser_null())
    if t == D.TIMER_TRIGGER:
        ty = r(0, 7)
        name = bytes(rng.integers(0x30, 0x7A, r(0, 90)).astype(np.uint8).tobytes()) if ty == D.INTERNAL else None
        return D.TimerTriggerDeterminant(r(0, 1 << 20), r(0, 1 << 45), ty, name)
    if t == D.SOURCE_CHECKPOINT:
        ref = None if r(0, 4) == 0 else bytes(rng.integers(0, 256, r(0, 120)).astype(np.uint8).tobytes())
        return D.SourceCheckpointDeterminant(r(0, 1 << 20), r(0, 1000), r(0, 1 << 45), r(0, 2), ref)
    return D.IgnoreCheckpointDeterminant(r(0, 1 << 20), r(0, 1000))


def random_log(n: int, rng: np.random.Generator, allow_serializable: bool = True) -> bytes:
    return b"".join(D.encode(random_determinant(rng, allow_serializable)) for _ in range(n))


SEED_CONFIG1 = 0xC105


def config1_job(rng: np.random.Generator, parallelism: int = 4, epoch_ms: int = 1000, checkpoints: int = 1):
    """Config 1 (BASELINE.json configs[0]): WordCount + causal TimeService with a
    processing-time window, parallelism 4, one epoch, modelled from the reference's producer
    call sites (a JVM MiniCluster capture cannot run here):
      every task's main log starts the epoch with Timestamp then RNG
        (subscription order StreamTask.java:305-313, EpochTrackerImpl.java:99-100);
      "PTS" TimerTrigger (21 B) every 5 ms of processing time (StreamTask.java:1519);
      source main logs: SourceCheckpoint (27 B) per checkpoint;
      window main logs: Order (2 B) per input buffer over 4 channels, window TimerTrigger
        "87" (20 B) per firing (WindowOperator.java:203);
      sink main logs: Order per input buffer;
      every subpartition log: BufferBuilt (5 B) per output buffer (PipelinedSubpartition).
    Returns (graph, {CausalLogID: bytes}) for stages source -> window -> sink."""
    from . import job
    from .engine import CausalLogID
    g = job.JobGraph([job.JobVertex("source", parallelism), job.JobVertex("window", parallelism, ["source"]),
                      job.JobVertex("sink", parallelism, ["window"])])
    logs = {}
    rc = 0
    for name in ("source", "window", "sink"):
        for i, vid in enumerate(g.vertex_ids(name)):
            recs = [D.TimestampDeterminant(1_700_000_000_000 + int(rng.integers(0, 1000))),
                    D.RNGDeterminant(int(rng.integers(-2**31, 2**31)))]
            t, n_in = 0, 0
            while t < epoch_ms:
                step = int(rng.integers(1, 6))
                t += step
                if name != "source":
                    for _ in range(int(rng.integers(0, 4))):
                        recs.append(D.OrderDeterminant(int(rng.integers(0, parallelism))))
                        n_in += 1
                if t % 5 < step:
                    recs.append(D.TimerTriggerDeterminant(n_in, 1_700_000_000_000 + t, D.INTERNAL, b"PTS"))
                if name == "window" and t % 100 < step:
                    recs.append(D.TimerTriggerDeterminant(n_in, 1_700_000_000_000 + t, D.INTERNAL, b"87"))
                if name == "source" and checkpoints and t % (epoch_ms // checkpoints) < step:
                    rc += 1
                    recs.append(D.SourceCheckpointDeterminant(rc, rc, 1_700_000_000_000 + t, D.CHECKPOINT, b""))
            logs[CausalLogID.main(vid)] = b"".join(D.encode(r) for r in recs)
            if name != "sink":
                for j in range(parallelism):  # one subpartition per downstream subtask
                    n = int(rng.integers(5, 200))
                    logs[CausalLogID.sub(vid, 0x5EED0000 + vid, 1, j)] = b"".join(
                        D.encode(D.BufferBuiltDeterminant(int(x))) for x in rng.integers(1, 32768, n))
    return g, logs
