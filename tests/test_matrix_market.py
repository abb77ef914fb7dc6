"""Matrix Market input for the SpMV workload (the reference vendors cwpearson/mm but never calls
it; here any square matrix file can replace the random band matrix)."""
import json

import pytest


def _write(path, text):
    path.write_text(text)
    return str(path)


def test_roundtrip_band_matrix(tz, tmp_path):
    rp, ci, v = tz._tz.random_band_matrix(300, 40, 3000, 7)
    f = str(tmp_path / "a.mtx")
    tz._tz.write_matrix_market(300, 300, rp, ci, v, f)
    rows, cols, rp2, ci2, v2 = tz._tz.read_matrix_market(f)
    assert (rows, cols) == (300, 300)
    assert list(rp2) == list(rp) and list(ci2) == list(ci)
    assert max(abs(a - b) for a, b in zip(v, v2)) < 1e-6


def test_symmetric_pattern_and_duplicates(tz, tmp_path):
    f = _write(tmp_path / "s.mtx", "%%MatrixMarket matrix coordinate real symmetric\n"
               "% a comment\n3 3 4\n1 1 2.0\n2 1 -1.5\n3 2 4\n3 2 1\n")
    rows, cols, rp, ci, v = tz._tz.read_matrix_market(f)
    dense = [[0.0] * 3 for _ in range(3)]
    for r in range(3):
        for j in range(rp[r], rp[r + 1]):
            dense[r][ci[j]] = v[j]
    # (3,2) appears twice: duplicates add up; the upper triangle mirrors the lower one
    assert dense == [[2.0, -1.5, 0.0], [-1.5, 0.0, 5.0], [0.0, 5.0, 0.0]]
    f = _write(tmp_path / "p.mtx", "%%MatrixMarket matrix coordinate pattern general\n2 2 2\n1 2\n2 1\n")
    _, _, rp, ci, v = tz._tz.read_matrix_market(f)
    assert list(rp) == [0, 1, 2] and list(ci) == [1, 0] and list(v) == [1.0, 1.0]
    f = _write(tmp_path / "k.mtx", "%%MatrixMarket matrix coordinate real skew-symmetric\n2 2 1\n2 1 3\n")
    _, _, rp, ci, v = tz._tz.read_matrix_market(f)
    assert list(ci) == [1, 0] and list(v) == [-3.0, 3.0]


@pytest.mark.parametrize("text,err", [
    ("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n", "coordinate"),
    ("%%MatrixMarket matrix coordinate complex general\n1 1 1\n1 1 1 0\n", "field"),
    ("%%MatrixMarket matrix coordinate real general\n2 2 1\n3 1 1.0\n", "out of range"),
    ("%%MatrixMarket matrix coordinate real general\n2 2 2\n1 1 1.0\n", "entries"),
    ("hello\n", "Matrix Market"),
    # more stored entries than int32 row pointers hold (checked before any entry is read)
    ("%%MatrixMarket matrix coordinate real symmetric\n10 10 1500000000\n1 1 1.0\n", "int32"),
])
def test_bad_files_are_rejected(tz, tmp_path, text, err):
    with pytest.raises(Exception, match=err):
        tz._tz.read_matrix_market(_write(tmp_path / "bad.mtx", text))


def test_spmv_workload_from_file_partitions_every_entry(tz, tmp_path):
    """row partition over 3 ranks: local + remote blocks of all ranks hold every nonzero once;
    a non-square matrix is refused"""
    from tenzing_amd.models import SpmvConfig

    n = 500
    rp, ci, v = tz._tz.random_band_matrix(n, 60, 5000, 3)
    f = str(tmp_path / "m.mtx")
    tz._tz.write_matrix_market(n, n, rp, ci, v, f)
    total = 0
    for r in range(3):
        s = tz._tz.DistSpmv(SpmvConfig(matrix=f).args(r, 3, -1))
        assert s.args.m == n
        total += s.local_nnz() + s.remote_nnz()
    assert total == rp[-1]
    g = tz.Graph()
    s.add_to_graph(g)
    seq = tz.random_rollout(tz.State(g, tz.Platform(2)), 0)
    assert len(seq) > 2
    bad = _write(tmp_path / "r.mtx", "%%MatrixMarket matrix coordinate real general\n2 3 1\n1 3 1\n")
    with pytest.raises(Exception, match="square"):
        tz._tz.DistSpmv(SpmvConfig(matrix=bad).args(0, 1, -1))


@pytest.mark.parametrize("ranks", [1, 4, 8])
def test_band_matrix_parity_with_the_reference_generator(tz, ranks):
    """the reference driver's matrix (spmv_run_strategy.cuh:67-68: m = 150,000, bw = m / ranks,
    nnz = 10 m) has exactly nnz distinct entries, all with |c - r| <= bw (csr_mat.hpp:334-370:
    refilled after duplicates are removed; columns drawn in [r - bw, r + bw])"""
    import numpy as np

    m = 150_000
    bw = m // ranks
    rp, ci, v = tz._tz.random_band_matrix(m, bw, 10 * m, 1)
    rp, ci = np.asarray(rp, dtype=np.int64), np.asarray(ci, dtype=np.int64)
    assert len(ci) == 10 * m and rp[-1] == 10 * m and len(v) == 10 * m
    rows = np.repeat(np.arange(m), np.diff(rp))
    assert np.abs(ci - rows).max() <= bw
    assert (ci >= 0).all() and (ci < m).all()
    # distinct (row, column) pairs, columns sorted within each row
    key = rows * m + ci
    assert (np.diff(key) > 0).all()


def test_spmv_workload_records_its_actual_nnz(tz):
    """every rank builds the same matrix; the args say how many entries it has, and the ranks'
    local + remote blocks partition exactly those"""
    from tenzing_amd.models import SpmvConfig

    total = 0
    for r in range(4):
        s = tz._tz.DistSpmv(SpmvConfig(m=20_000).args(r, 4, -1))
        assert s.args.nnz_actual == 200_000
        assert json.loads(s.args.json())["nnz_actual"] == 200_000
        total += s.local_nnz() + s.remote_nnz()
    assert total == 200_000


def test_band_matrix_rejects_more_entries_than_the_band_holds(tz):
    with pytest.raises(Exception, match="exceeds"):
        tz._tz.random_band_matrix(10, 1, 29, 1)  # 3 per row, minus the 2 corners: 28
    rp, ci, _ = tz._tz.random_band_matrix(10, 1, 28, 1)
    assert len(ci) == 28
