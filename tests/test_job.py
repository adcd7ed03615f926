"""CPU: job-level sharing-depth bookkeeping (clonos_amd/job.py) against hand-derived
expectations from the reference algorithms (CausalGraphUtils.java:43-123,
AbstractDeltaSerializerDeserializer.java:177, JobCausalLogImpl.java:136-204)."""
import pytest

from clonos_amd import job as J


def diamond():
    # src -> (a, b) -> sink ; parallelism 2, 1, 3, 2
    return J.JobGraph([J.JobVertex("src", 2), J.JobVertex("a", 1, ["src"]), J.JobVertex("b", 3, ["src"]),
                       J.JobVertex("sink", 2, ["a", "b"])])


def test_vertex_ids():
    g = diamond()
    assert g.vertex_ids("src") == [0, 1]
    assert g.vertex_ids("a") == [2]
    assert g.vertex_ids("b") == [3, 4, 5]
    assert g.vertex_ids("sink") == [6, 7]
    # the counter is a Java short: it wraps
    big = J.JobGraph([J.JobVertex("x", 40000), J.JobVertex("y", 2, ["x"])])
    assert big.vertex_id("y", 1) == ((40001 + 0x8000) & 0xFFFF) - 0x8000


def test_distances_diamond():
    g = diamond()
    d = g.distances("sink")
    assert d == {6: 0, 7: 0, 2: -1, 3: -1, 4: -1, 5: -1, 0: -2, 1: -2}
    d = g.distances("a")
    assert d == {2: 0, 0: -1, 1: -1, 6: 1, 7: 1}  # b is unrelated to a: absent
    d = g.distances("src")
    assert d[6] == 2 and d[3] == 1 and d[0] == 0


def test_distances_shortest_path_wins():
    # src -> mid -> sink and src -> sink: src is at distance -1 from sink (max merge)
    g = J.JobGraph([J.JobVertex("src", 1), J.JobVertex("mid", 1, ["src"]), J.JobVertex("sink", 1, ["mid", "src"])])
    assert g.distances("sink") == {2: 0, 1: -1, 0: -1}
    assert g.distances("src") == {0: 0, 1: 1, 2: 1}  # downstream min merge


def test_sharing_rules():
    assert not J.shares_local_logs(0) and J.shares_local_logs(1) and J.shares_local_logs(-1)
    assert J.shares_upstream_log(-1, 2) and not J.shares_upstream_log(-2, 2) and J.shares_upstream_log(-9, -1)
    assert J.answers_request(-2, 2) and not J.answers_request(-3, 2) and J.answers_request(5, -1)


@pytest.mark.parametrize("depth,expect", [(0, set()), (1, {2, 3, 4, 5}), (2, {0, 1, 2, 3, 4, 5}), (-1, {0, 1, 2, 3, 4, 5})])
def test_held_upstream(depth, expect):
    assert J.held_upstream_vertices(diamond(), "sink", depth) == expect


def test_config4_replication_plan():
    """5-stage DAG, parallelism 128, full sharing, 8 GPUs: 640 VertexIDs; a rank needs
    every upstream log of every stage it hosts, minus the ones it owns."""
    g = J.dag(5, 128)
    ids = [vid for _, _, vid in g.all_vertex_ids()]
    assert ids == list(range(640))
    plan = J.replication_plan(g, -1, 8)
    for r in range(8):
        # rank r hosts subtasks of stages 1..4, so it needs all of stages 0..3 not owned by r
        assert plan[r] == {v for v in range(512) if v % 8 != r}
    plan1 = J.replication_plan(g, 1, 8)
    assert plan1[0] == {v for v in range(512) if v % 8 != 0}  # depth 1: direct producers only
    plan_local = J.replication_plan(g, 0, 8)
    assert all(not s for s in plan_local.values())


def test_responders():
    g = diamond()
    # failed 'a' (vid 2): depth 1 -> its direct neighbours answer (src and sink subtasks)
    assert sorted(J.responders(g, 2, 1)) == [0, 1, 6, 7]
    # failed src (vid 0): a, b and its sibling subtask 1 (distance 0, answers with no logs of 0)
    assert sorted(J.responders(g, 0, 1)) == [1, 2, 3, 4, 5]
    assert sorted(J.responders(g, 0, -1)) == [1, 2, 3, 4, 5, 6, 7]  # src's sibling subtask is at distance 0
