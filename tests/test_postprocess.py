"""Design-rule mining on synthetic search results (reference postprocess/postprocess.py)."""
import numpy as np

from test_core import diamond


def test_classes_and_rules(tz, tmp_path):
    from tenzing_amd.utils import postprocess as pp

    g = diamond(tz, a=10, b=200, c=200, d=10)
    p = tz.SimParams()
    p.launch_us = 1.0
    o = tz.DfsOpts()
    o.bench = tz.BenchOpts(n_iters=2)
    r = tz.dfs_explore(g, tz.Platform(2), tz.SimBenchmarker(2, p), tz.SelfCtrl(), o)
    path = tmp_path / "r.csv"
    path.write_text(r.dump_csv())
    res = pp.load_results(str(path))
    assert len(res) == len(r.sims)
    labels, bounds = pp.performance_classes([x.pct10 for x in res])
    assert labels.max() >= 1  # overlapped (k2 || k3) vs serialized schedules
    report, rules = pp.process(res)
    assert report["classes"] >= 2 and rules
    text = pp.format_rules(rules, report)
    assert "same stream" in text  # the rule is about k2/k3 sharing a stream
    # JSONL input works too
    pj = tmp_path / "r.jsonl"
    pj.write_text(r.dump_jsonl())
    assert len(pp.load_results(str(pj))) == len(res)
    acc = pp.evaluate_rules(res, max(4, len(res) // 2))
    assert acc is None or 0.0 <= acc <= 1.0


def test_peaks_on_step_data():
    from tenzing_amd.utils import postprocess as pp

    t = np.concatenate([np.full(50, 1.0), np.full(50, 2.0), np.full(50, 3.0)])
    rng = np.random.default_rng(0)
    t = t + rng.normal(0, 0.01, t.size)
    labels, bounds = pp.performance_classes(t, radius_frac=0.02, pctl=95)
    assert len(set(labels)) == 3


def test_rules_cli_writes_the_reference_figures(tz, tmp_path):
    """`rules --plots`: the class figure (sorted times, step response, boundaries), the decision
    tree and the accuracy-vs-training-size figure, as the reference's postprocess.py draws"""
    from tenzing_amd.utils import postprocess as pp

    g = diamond(tz, a=10, b=200, c=200, d=10)
    o = tz.DfsOpts()
    o.bench = tz.BenchOpts(n_iters=2)
    r = tz.dfs_explore(g, tz.Platform(2), tz.SimBenchmarker(2, tz.SimParams()), tz.SelfCtrl(), o)
    path = tmp_path / "r.csv"
    path.write_text(r.dump_csv())
    prefix = str(tmp_path / "d_")
    assert pp.main([str(path), "--out", prefix, "--plots", "--eval", "4", "8"]) == 0
    for name in ("classes.pdf", "tree.pdf", "eval.pdf", "rules.txt", "classes.json"):
        f = tmp_path / ("d_" + name)
        assert f.exists() and f.stat().st_size > 0, name
    assert (tmp_path / "d_classes.pdf").read_bytes()[:4] == b"%PDF"
