"""The driver's one-GPU bench command end to end, with what it records after the headline: the
graph-branch probe and the stream padding it chose, the reference driver's XYZQ layout and
BASELINE configs 2 (SpMV) and 5 (SpMV + halo) as searched, verified and timed sub-records, and
the post-timing budget (a stalled sub-record costs neither the headline nor the exit status)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(extra, env=None, timeout=200):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cells", "64", "--mcts-iters", "6",
           "--steps", "5", "--warmup", "2"] + extra
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout,
                       env=dict(os.environ, **(env or {})))
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    return r, lines


def test_bench_one_rank_subrecords(gpu):
    r, lines = _bench([])
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j["partial"] is False and j["verified_bad_cells"] == 0 and j["value"] > 0
    # the padding the search ran with, and whether 3 graph branches ran at once with it
    bp = j["graph_branch_probe"]
    assert bp["tried"] and bp["tried"][0]["probe"]["ratio"] > 0, bp
    assert bp["tried"][0]["probe"]["unrolled"]["ratio"] > 0, bp
    assert j["pad_streams"] == bp["pad_streams"]
    assert j["post_timing"]["done"] == ["torch_model", "move_roof", "reference_layout", "baseline_configs"]
    assert j["torch_model_check"]["bad_cells"] == 0, j["torch_model_check"]
    for roof in (j["move_roof"], j["reference_layout"]["move_roof"]):
        assert roof["move_us"] > 0 and roof["roof_us"] > 0 and roof["read_lines_MB"] > 0, roof
    ref = j["reference_layout"]
    assert "error" not in ref, ref
    assert ref["verified_bad"] == 0 and ref["verified_bad_after_timing"] == 0
    assert ref["ms_per_step"] > 0 and ref["steps"] == 5
    lay = ref["config"]["layout"]
    # the reference's storage: x = 0 at the row start, rows padded to 128 B (64 + 6 -> 80)
    assert lay["order"] == "xyzq" and lay["x_offset_cells"] == 0 and lay["row_pitch_elems"] == 80
    # the x faces of one row moved together (their ghost and source runs share a line)
    assert ref["move_roof"]["pairs"] == 1
    for name in ("spmv_c2", "fused_c5"):
        rec = j["baseline_configs"][name]
        assert "error" not in rec, rec
        assert rec["verified_bad"] == 0 and rec["verified_bad_after_timing"] == 0, rec
        assert rec["ms_per_step"] > 0 and rec["mcts_candidates"] > 0
    assert j["baseline_configs"]["spmv_c2"]["config"]["nnz"] == 1_500_000


def test_bench_one_rank_stall_after_headline(gpu):
    """the first sub-record never returns: the complete line is printed by the post-timing
    budget, with exit status 0, naming the sub-record that did not finish"""
    r, lines = _bench(["--post-budget-s", "8", "--branch-probe", "off"],
                      env={"TZ_BENCH_STALL": "reference_layout"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1
    j = json.loads(lines[0])
    assert j["partial"] is False and j["phase"] == "done" and j["verified_bad_cells"] == 0
    assert j["post_timing"]["running"] == "reference_layout" and "reference_layout" not in j
    assert j["graph_branch_probe"] is None
