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


@st.composite
def nested_dags(draw):
    """a random DAG whose vertices may be choices of 2-3 alternatives or compounds of a small
    chain (one level of nesting, plus a choice inside a compound)"""
    n, gpu, edges = draw(dags())
    kinds = draw(st.lists(st.sampled_from(["op", "choice", "compound"]), min_size=n, max_size=n))
    alts = draw(st.lists(st.integers(min_value=2, max_value=3), min_size=n, max_size=n))
    return n, gpu, edges, kinds, alts


def build_nested(tz, n, gpu, edges, kinds, alts):
    def leaf(name, i):
        return tz.SimGpuOp(name, 10.0 + i) if gpu[i] else tz.SleepOp(name, 0.0)

    ops = []
    for i in range(n):
        if kinds[i] == "choice":
            ops.append(tz.StaticChoiceOp(f"ch{i}", [leaf(f"ch{i}_{a}", i) for a in range(alts[i])]))
        elif kinds[i] == "compound":
            sub = tz.Graph()
            a, b = tz.SimGpuOp(f"cp{i}_a", 5.0), tz.StaticChoiceOp(
                f"cp{i}_b", [tz.SimGpuOp(f"cp{i}_b{k}", 5.0 + k) for k in range(alts[i])])
            sub.start_then(a)
            sub.then(a, b)
            sub.then_finish(b)
            ops.append(tz.StaticCompoundOp(f"cp{i}", sub))
        else:
            ops.append(leaf(f"v{i}", i))
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


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(dag=nested_dags(), streams=st.integers(min_value=1, max_value=4),
       seed=st.integers(min_value=0, max_value=2**31 - 1))
def test_loaded_schedules_verify_on_the_resolved_graph(tz, dag, streams, seed):
    """any schedule of a graph with choices and compounds, read back from its JSON, is race-free
    on resolve_graph(graph, schedule), which has no choice or compound left"""
    g = build_nested(tz, *dag)
    seq = tz.random_rollout(tz.State(g, tz.Platform(streams)), seed)
    back = tz.OpIndex(g).sequence_from_json(seq.json(True))
    fg = tz.resolve_graph(g, back)
    kinds = {fg.op(v).kind for v in fg.vertices()}
    assert not kinds & {"ChoiceOp", "CompoundOp"}, kinds
    assert tz.verify(back, fg, streams) == []
