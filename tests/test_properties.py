"""Property tests of the synchronizer over random op DAGs (no GPU).

SURVEY.md §4 lists "no synchronizer race-freedom property test" among the reference's test gaps;
the reference's own checks are fixed graphs (test/test_noop_graph.cpp, test/test_gpu_graph.cu).
Here hypothesis draws DAGs of simulated GPU ops and host ops with random edges, and for every
random schedule of them over 1-4 streams checks:

* the schedule is race-free under the vector-clock checker (`verify`);
* it survives a JSON round trip through `OpIndex` (schedule schema, §2.7);
* `remove_redundant_syncs` keeps it race-free and leaves a minimal sync set: dropping any one
  remaining wait/sync op makes `verify` report a violation.
"""
import json

import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

WAIT_KINDS = {"CudaStreamWaitEvent", "CudaEventSync", "StreamWait", "StreamSync"}


@st.composite
def dags(draw):
    n = draw(st.integers(min_value=1, max_value=6))
    gpu = draw(st.lists(st.booleans(), min_size=n, max_size=n))
    edges = [(i, j) for j in range(n) for i in range(j)
             if draw(st.integers(min_value=0, max_value=2)) == 0]
    return n, gpu, edges


def build(tz, n, gpu, edges):
    ops = [tz.SimGpuOp(f"g{i}", 10.0 + i) if gpu[i] else tz.SleepOp(f"c{i}", 0.0)
           for i in range(n)]
    g = tz.Graph()
    has_pred = {j for _, j in edges}
    has_succ = {i for i, _ in edges}
    for i in range(n):
        if i not in has_pred:
            g.start_then(ops[i])
    for i, j in edges:
        g.then(ops[i], ops[j])
    for i in range(n):
        if i not in has_succ:
            g.then_finish(ops[i])
    return g


def without(tz, seq, k):
    out = tz.Sequence()
    for i, op in enumerate(seq.ops()):
        if i != k:
            out.append(op)
    return out


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(dag=dags(), streams=st.integers(min_value=1, max_value=4),
       seed=st.integers(min_value=0, max_value=2**31 - 1))
def test_random_dag_schedules_race_free_and_minimal(tz, dag, streams, seed):
    g = build(tz, *dag)
    ng = g.clone()
    ng.normalize()
    seq = tz.random_rollout(tz.State(g, tz.Platform(streams)), seed)
    assert tz.verify(seq, ng, streams) == []

    back = tz.OpIndex(g).sequence_from_json(seq.json(True))
    assert back.canonical_key() == seq.canonical_key()

    pruned, k = tz.remove_redundant_syncs(seq, ng, streams)
    assert len(pruned) == len(seq) - k
    assert tz.verify(pruned, ng, streams) == []
    for i, op in enumerate(pruned.ops()):
        if json.loads(op.json()).get("kind") in WAIT_KINDS:
            assert tz.verify(without(tz, pruned, i), ng, streams) != [], (
                f"sync {i} of {pruned.desc()} is redundant")
