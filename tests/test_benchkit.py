"""bench.py's testable pieces on the CPU: the stream-padding choice driven by the graph-branch
probe (fake runtimes and a fake timer), and the run deadline's post-headline budget (a stall
after the result is final still prints the complete line and exits 0)."""
import json
import os
import subprocess
import sys

from tenzing_amd.utils.benchkit import choose_pad

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeRt:
    made = []

    def __init__(self, pad):
        self.pad_streams = 6 if pad is None else pad
        FakeRt.made.append(self.pad_streams)


def fake_probe(ratios):
    """the probe's ratio per padding (None: the probe could not run)"""
    def probe(rt):
        r = ratios[rt.pad_streams]
        return None if r is None else {"ratio": r, "one_us": 55.0, "all_us": 55.0 * r}
    return probe


def test_choose_pad_keeps_the_default_when_branches_run_at_once():
    FakeRt.made = []
    rt, rec = choose_pad(FakeRt, fake_probe({6: 1.1, 8: 1.0}), [None, 8, 12])
    assert rt.pad_streams == 6 and rec["pad_streams"] == 6 and rec["serialized"] is False
    assert FakeRt.made == [6] and len(rec["tried"]) == 1


def test_choose_pad_retries_until_a_padding_runs_branches_at_once():
    FakeRt.made = []
    rt, rec = choose_pad(FakeRt, fake_probe({6: 2.05, 8: 1.9, 12: 1.15, 4: 1.0}), [None, 8, 12, 4])
    assert rt.pad_streams == 12 and rec["serialized"] is False
    assert [t["pad_streams"] for t in rec["tried"]] == [6, 8, 12]
    assert FakeRt.made == [6, 8, 12]


def test_choose_pad_falls_back_to_the_least_serialized():
    FakeRt.made = []
    rt, rec = choose_pad(FakeRt, fake_probe({6: 2.0, 8: 1.7, 12: 1.9, 4: 2.1}), [None, 8, 12, 4])
    # none within the threshold: the lowest ratio (8, clearly below the default's) is rebuilt
    # and recorded as serialized
    assert rt.pad_streams == 8 and rec["pad_streams"] == 8 and rec["serialized"] is True
    assert FakeRt.made == [6, 8, 12, 4, 8]


def test_choose_pad_keeps_the_default_when_no_padding_is_clearly_better():
    """every padding serializes alike (probe noise apart): the default stays"""
    FakeRt.made = []
    rt, rec = choose_pad(FakeRt, fake_probe({6: 1.67, 8: 1.634, 12: 1.629, 4: 1.637}), [None, 8, 12, 4])
    assert rt.pad_streams == 6 and rec["serialized"] is True
    assert FakeRt.made == [6, 8, 12, 4, 6]


def test_choose_pad_judges_the_unrolled_ratio_when_the_probe_has_it():
    """one copy per launch looks serialized (launch-boundary stagger), the unrolled graph the
    search replays runs the branches at once: the default padding stays"""
    FakeRt.made = []

    def probe(rt):
        return {"ratio": 1.9, "unrolled": {"ratio": 1.05 if rt.pad_streams == 6 else 1.0}}
    rt, rec = choose_pad(FakeRt, probe, [None, 8, 12, 4])
    assert rt.pad_streams == 6 and rec["serialized"] is False and FakeRt.made == [6]


def test_choose_pad_when_the_probe_cannot_run():
    FakeRt.made = []
    rt, rec = choose_pad(FakeRt, fake_probe({6: None, 8: None}), [None, 8])
    assert rec["serialized"] is None and rt.pad_streams == 8 and FakeRt.made == [6, 8]


def _run(code, timeout=60):
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=timeout, cwd=ROOT)


def test_deadline_tighten_prints_the_final_line_and_exits_0():
    """the bench's post-headline phase: the report is the complete (non-partial) line, the
    deadline is tightened to the post budget with exit status 0, and a diagnostic then stalls:
    the line is printed once and the process exits 0 within the budget"""
    code = ("import json, time, tenzing_amd as tz\n"
            "d = tz.RunDeadline(300.0, 5)\n"
            "d.set_report(json.dumps({'metric': 'm', 'value': 0.1, 'partial': True}))\n"
            "d.set_report(json.dumps({'metric': 'm', 'value': 0.2, 'partial': False,\n"
            "                         'post_timing': {'running': 'link_matrix'}}))\n"
            "d.tighten(1.0, 0)\n"
            "time.sleep(60)\n")
    r = _run(code)
    assert r.returncode == 0, (r.stdout, r.stderr)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j["partial"] is False and j["value"] == 0.2
    assert j["post_timing"]["running"] == "link_matrix"
    assert "run deadline" in r.stderr and "status 0" in r.stderr


def test_deadline_tighten_never_extends():
    """tighten() can only bring the deadline closer: a later instant keeps the earlier one (its
    exit status is still replaced)"""
    code = ("import time, tenzing_amd as tz\n"
            "d = tz.RunDeadline(1.0, 5)\n"
            "d.set_report('{\"v\": 1}')\n"
            "d.tighten(100.0, 7)\n"
            "assert d.remaining < 1.5\n"
            "time.sleep(30)\n")
    r = _run(code)
    assert r.returncode == 7, (r.stdout, r.stderr)


def test_deadline_cancel_after_tighten():
    code = ("import time, tenzing_amd as tz\n"
            "d = tz.RunDeadline(30.0, 5)\n"
            "d.tighten(0.5, 0)\n"
            "d.cancel()\n"
            "time.sleep(1.2)\n"
            "print('alive')\n")
    r = _run(code)
    assert r.returncode == 0 and "alive" in r.stdout, (r.stdout, r.stderr)


def test_scale_report_rows(tmp_path):
    """the per-GPU-count table: the final line of each run (partial lines skipped), the floor
    the run's own link probe gives, weak-scaling efficiency against the N=1 record"""
    from tenzing_amd.utils.scale_report import records, rows

    def rec(n, ms, partial=False, **kw):
        return json.dumps({"metric": "m", "value": ms, "n_gpus": n, "partial": partial,
                           "config": {"rank_grid": [1, 1, n]}, **kw})

    (tmp_path / "n1.jsonl").write_text(rec(1, 0.09, True) + "\n" + rec(1, 0.045) + "\n")
    (tmp_path / "n2.jsonl").write_text(rec(2, 0.4, link_probe={
        "GBps": {"put": 70.0}, "busiest_link_at_probe_rate_ms": 0.25},
        model_check={"spearman": 0.9}) + "\n")
    rs = rows(records([str(tmp_path / "n2.jsonl"), str(tmp_path / "n1.jsonl")]))
    assert [r["n_gpus"] for r in rs] == [1, 2] and rs[0]["ms"] == 0.045
    assert rs[1]["ms_over_link_floor"] == 1.6 and rs[1]["model_spearman"] == 0.9
    assert rs[1]["weak_efficiency"] == round(0.045 / 0.4, 3)
    out = subprocess.run([sys.executable, "-m", "tenzing_amd.utils.scale_report",
                          str(tmp_path / "n1.jsonl"), str(tmp_path / "n2.jsonl")],
                         capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode == 0 and "ms_over_link_floor" in out.stdout, out.stderr
