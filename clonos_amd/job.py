"""Job-level causal-log bookkeeping: vertex IDs, graph distances and the sharing-depth
rules that decide which (consumer, log) pairs get delta slices, which logs a task keeps,
and which tasks answer a determinant request.

Host logic only (integer graph work on small job graphs); the byte work it schedules
runs in the engine.  Reference (R/ = flink-runtime/src/main/java/org/apache/flink/runtime/causal/):
  computeVertexId        R/CausalGraphUtils.java:43-54
  computeDistances       R/CausalGraphUtils.java:88-123 (BFS, upstream max-merge negative,
                         downstream min-merge positive; unrelated vertices absent)
  insertNewUpstreamLog   R/log/job/serde/AbstractDeltaSerializerDeserializer.java:165-194 (:177)
  registerTask           R/log/job/JobCausalLogImpl.java:125-169 (local logs shared iff depth != 0)
  respondToDeterminantRequest  R/log/job/JobCausalLogImpl.java:188-204
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Sequence, Set, Tuple

import numpy as np

FULL_SHARING = -1  # ExecutionConfig.determinantSharingDepth default


@dataclass
class JobVertex:
    """A job vertex: name (JobVertexID), parallelism and the producers of its inputs."""
    name: str
    parallelism: int
    inputs: List[str] = field(default_factory=list)


class JobGraph:
    """Job vertices in topological order (the `sortedJobVertexes` list of the reference)."""

    def __init__(self, vertices: Sequence[JobVertex]):
        self.vertices = list(vertices)
        self.by_name = {v.name: v for v in self.vertices}
        if len(self.by_name) != len(self.vertices):
            raise ValueError("duplicate job vertex names")
        seen: Set[str] = set()
        for v in self.vertices:
            for p in v.inputs:
                if p not in seen:
                    raise ValueError(f"vertices not topologically sorted: {v.name} before its input {p}")
            seen.add(v.name)
        self.consumers: Dict[str, List[str]] = {v.name: [] for v in self.vertices}
        for v in self.vertices:
            for p in dict.fromkeys(v.inputs):  # distinct producers
                self.consumers[p].append(v.name)

    # ---- CausalGraphUtils.computeVertexId :43-54 -------------------------------------
    def vertex_id(self, name: str, subtask: int) -> int:
        """Sum of the parallelism of earlier vertices + subtaskIndex, as a Java `short`."""
        c = 0
        for v in self.vertices:
            if v.name == name:
                c += subtask
                break
            c += v.parallelism
        return ((c + 0x8000) & 0xFFFF) - 0x8000

    def vertex_ids(self, name: str) -> List[int]:
        return [self.vertex_id(name, i) for i in range(self.by_name[name].parallelism)]

    def all_vertex_ids(self) -> List[Tuple[str, int, int]]:
        """(job vertex, subtask, VertexID) for every subtask, in VertexID order."""
        return [(v.name, i, self.vertex_id(v.name, i)) for v in self.vertices for i in range(v.parallelism)]

    # ---- CausalGraphUtils.computeDistances :88-123 ---------------------------------------
    def _bfs(self, dist: Dict[int, int], start: str, explore, merge) -> None:
        todo = deque([(0, start)])  # ArrayDeque: push() = addFirst, addAll = addLast, pop() = removeFirst
        while todo:
            d, name = todo.popleft()
            distance = 0
            for vid in self.vertex_ids(name):
                distance = merge(dist[vid], d) if vid in dist else d
                dist[vid] = distance
            todo.extend(explore(name, distance))

    def distances(self, name: str) -> Dict[int, int]:
        """VertexID -> signed distance from job vertex `name` (upstream < 0 < downstream)."""
        dist: Dict[int, int] = {}
        self._bfs(dist, name, lambda n, d: [(d - 1, p) for p in dict.fromkeys(self.by_name[n].inputs)], max)
        self._bfs(dist, name, lambda n, d: [(d + 1, c) for c in self.consumers[n]], min)
        return dist


# ---- sharing-depth rules ----------------------------------------------------------------
def shares_local_logs(depth: int) -> bool:
    """registerTask :136-169: a task's own logs are shared downstream iff depth != 0."""
    return depth != 0


def shares_upstream_log(distance: int, depth: int) -> bool:
    """insertNewUpstreamLog :177: an upstream log is shared further iff depth == -1 or
    |distance| + 1 <= depth."""
    return depth == FULL_SHARING or abs(distance) + 1 <= depth


def answers_request(distance: int, depth: int) -> bool:
    """respondToDeterminantRequest :192: answer iff depth == -1 or |distance| <= depth."""
    return depth == FULL_SHARING or abs(distance) <= depth


def held_upstream_vertices(graph: JobGraph, name: str, depth: int) -> Set[int]:
    """VertexIDs whose logs a subtask of job vertex `name` holds replicas of.

    A producer p piggybacks its own logs (depth != 0) and the upstream logs it shares
    (|dist(u, p)| + 1 <= depth); following that rule along every path, a task holds the
    logs of the upstream vertices within `depth` hops (all of them at full sharing).
    Depends on the job vertex only, not on the subtask."""
    if depth == 0:
        return set()
    return {vid for vid, d in graph.distances(name).items() if d < 0 and (depth == FULL_SHARING or -d <= depth)}


# ---- multi-GPU placement ----------------------------------------------------
def owner_rank(vertex_id: int, world: int) -> int:
    """Logs shard by VertexID: GPU g owns the vertices v with v mod G == g."""
    return (vertex_id & 0xFFFF) % world


def held_table(graph: JobGraph, depth: int) -> Dict[str, np.ndarray]:
    """job vertex -> sorted VertexIDs its subtasks hold replicas of (one BFS per job
    vertex: computeDistances depends on the job vertex only)."""
    return {v.name: np.array(sorted(held_upstream_vertices(graph, v.name, depth)), np.int64)
            for v in graph.vertices}


def replication_plan(graph: JobGraph, depth: int, world: int) -> Dict[int, Set[int]]:
    """rank -> VertexIDs owned by OTHER ranks whose logs that rank must receive (the
    union of the replicas its local subtasks hold)."""
    need = replication_masks(graph, depth, world)
    return {r: set(np.nonzero(need[r])[0].tolist()) for r in range(world)}


def replication_masks(graph: JobGraph, depth: int, world: int) -> np.ndarray:
    """bool[world, n_vertices]: [r, v] iff rank r needs replicas of vertex v's logs (v is
    held upstream by a subtask placed on r and owned by another rank).  Vectorised over
    VertexIDs (the reference's VertexIDs are 0 .. total parallelism - 1)."""
    ids = graph.all_vertex_ids()
    n = len(ids)
    held = held_table(graph, depth)
    owner = np.array([owner_rank(v, world) for _, _, v in ids], np.int64)
    need = np.zeros((world, n), bool)
    for v in graph.vertices:
        h = held[v.name]
        if h.size == 0:
            continue
        vids = np.array(graph.vertex_ids(v.name), np.int64)
        for r in np.unique(owner[vids]):
            need[r, h] = True
    need &= owner[None, :] != np.arange(world)[:, None]
    return need


def task_logs(graph: JobGraph, name: str, subtask: int):
    """The CausalLogIDs a subtask creates (registerTask :125-169): its main-thread log and,
    per output IntermediateResultPartition (one per consuming job vertex, produced by this
    subtask), one log per subpartition (= the consumer's parallelism).  The partition ID is
    synthetic but stable: lower = VertexID << 16 | output index, upper = 0xC105."""
    from .engine import CausalLogID
    vid = graph.vertex_id(name, subtask)
    out = [CausalLogID.main(vid)]
    for k, c in enumerate(graph.consumers[name]):
        lo = ((vid & 0xFFFF) << 16) | k
        out += [CausalLogID.sub(vid, lo, 0xC105, s) for s in range(graph.by_name[c].parallelism)]
    return out


class LogTable:
    """Every log of a job in one canonical order that all ranks agree on (VertexID order;
    per vertex: main log, then subpartition logs): the global log index `gid` replaces
    the CausalLogID on the replication wire and indexes dense per-rank handle tables."""

    def __init__(self, graph: JobGraph):
        self.graph = graph
        self.ids = []
        vert = []
        for name, sub, vid in graph.all_vertex_ids():
            for cid in task_logs(graph, name, sub):
                self.ids.append(cid)
                vert.append(vid)
        self.vertex = np.array(vert, np.int64)
        self._gid = {cid.key(): i for i, cid in enumerate(self.ids)}
        # each vertex's logs are one contiguous run of gids: vid -> (first, end)
        self._vrange = {}
        for i, v in enumerate(vert):
            a, _ = self._vrange.get(v, (i, i))
            self._vrange[v] = (a, i + 1)

    def gids_of(self, vertices) -> np.ndarray:
        """The gids of every log of these VertexIDs, ascending (np.nonzero(np.isin(vertex, vertices)),
        from the per-vertex runs: O(logs returned), not O(table))."""
        rs = [self._vrange[int(v)] for v in set(int(x) for x in vertices) if int(v) in self._vrange]
        if not rs:
            return np.zeros(0, np.int64)
        rs.sort()
        return np.concatenate([np.arange(a, b, dtype=np.int64) for a, b in rs])

    def __len__(self):
        return len(self.ids)

    def gid(self, cid) -> int:
        return self._gid[cid.key()]


def dag(stages: int, parallelism: int) -> JobGraph:
    """A linear `stages`-stage job with all-to-all edges (config 4's 5-stage DAG)."""
    vs = [JobVertex(f"stage{i}", parallelism, [f"stage{i - 1}"] if i else []) for i in range(stages)]
    return JobGraph(vs)


def responders(graph: JobGraph, failed_vertex_id: int, depth: int,
               candidates: Optional[Iterable[Tuple[str, int, int]]] = None) -> List[int]:
    """VertexIDs of the subtasks that answer a DeterminantRequestEvent for the failed
    vertex (respondToDeterminantRequest :188-204) among `candidates` (default: all)."""
    out = []
    for name, _, vid in (candidates if candidates is not None else graph.all_vertex_ids()):
        d = graph.distances(name).get(failed_vertex_id)
        if d is not None and vid != failed_vertex_id and answers_request(d, depth):
            out.append(vid)
    return out
