"""Torch-facing kernel wrappers (tenzing_amd.ops) vs plain PyTorch references."""
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def test_ops_wrappers(tz, gpu):
    from tenzing_amd import ops

    n = 3000
    rp, ci, val = tz._tz.random_band_matrix(n, 200, 8 * n, 3)
    rp = torch.tensor(rp, dtype=torch.int32, device="cuda")
    ci = torch.tensor(ci, dtype=torch.int32, device="cuda")
    val = torch.tensor(val, dtype=torch.float32, device="cuda")
    x = torch.randn(n, device="cuda")
    y = ops.csr_spmv(rp, ci, val, x)
    A = torch.sparse_csr_tensor(rp.long(), ci.long(), val, size=(n, n)).to_dense()
    torch.testing.assert_close(y, A @ x, rtol=1e-4, atol=1e-4)
    a, b = torch.randn(1001, device="cuda"), torch.randn(1001, device="cuda")
    torch.testing.assert_close(ops.vector_add(a, b), a + b)
    idx = torch.randint(0, 1001, (64,), dtype=torch.int32, device="cuda")
    torch.testing.assert_close(ops.gather(a, idx), a[idx.long()])
    d = torch.empty_like(a)
    ops.copy_(d, a)
    torch.testing.assert_close(d, a)
    grid = torch.randn(10 * 12 * 7, dtype=torch.float64, device="cuda")
    box = dict(grid_off=3, s1=10, s2=120, s3=0, len=5, n1=4, n2=6, n3=1)
    buf = ops.box_pack(grid, box)
    ref = torch.stack([grid[3 + 120 * k + 10 * j: 3 + 120 * k + 10 * j + 5] for k in range(6) for j in range(4)])
    torch.testing.assert_close(buf, ref.reshape(-1))
    with pytest.raises(IndexError):
        ops.box_pack(grid, dict(box, n2=100))
    with pytest.raises(TypeError):
        ops.csr_spmv(rp, ci, val.double(), x)
