"""Numerics of the hand-written gfx950 kernels against plain PyTorch fp32/fp64 references."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("order", ["xyzq", "qxyz"])
@pytest.mark.parametrize("neighbors", [6, 26])
def test_box_copy_pack_unpack_matches_torch(tz, gpu, order, neighbors):
    a = tz.HaloArgs()
    a.nx, a.ny, a.nz, a.nq, a.ghost = 20, 12, 9, 3, 2
    a.neighbors, a.order = neighbors, order
    h = tz.HaloExchange(a)
    n = h.grid_elems()
    grid = torch.randn(n, dtype=torch.float64, device="cuda")
    X, Y, Z, g = a.nx + 2 * a.ghost, a.ny + 2 * a.ghost, a.nz + 2 * a.ghost, a.ghost
    for i in range(h.ndirs()):
        box = h.pack_box(i)
        cnt = box["len"] * box["n1"] * box["n2"] * box["n3"]
        buf = torch.zeros(cnt, dtype=torch.float64, device="cuda")
        box["buf"] = buf.data_ptr()
        tz._tz.kernels.box_copy(grid.data_ptr(), box, False, _stream())
        # torch reference: gather the same rows with strided views
        ref = torch.empty(box["n3"], box["n2"], box["n1"], box["len"], dtype=torch.float64, device="cuda")
        for i3 in range(box["n3"]):
            for i2 in range(box["n2"]):
                base = box["grid_off"] + i2 * box["s2"] + i3 * box["s3"]
                rows = grid.as_strided((box["n1"], box["len"]), (box["s1"], 1), base)
                ref[i3, i2] = rows
        torch.cuda.synchronize()
        assert torch.equal(buf, ref.reshape(-1)), f"pack mismatch dir {h.dir_name(i)}"
        # unpack into a copy and compare
        g2 = grid.clone()
        src = torch.randn(cnt, dtype=torch.float64, device="cuda")
        box["buf"] = src.data_ptr()
        tz._tz.kernels.box_copy(g2.data_ptr(), box, True, _stream())
        exp = grid.clone()
        srcv = src.view(box["n3"], box["n2"], box["n1"], box["len"])
        for i3 in range(box["n3"]):
            for i2 in range(box["n2"]):
                base = box["grid_off"] + i2 * box["s2"] + i3 * box["s3"]
                exp.as_strided((box["n1"], box["len"]), (box["s1"], 1), base).copy_(srcv[i3, i2])
        torch.cuda.synchronize()
        assert torch.equal(g2, exp), f"unpack mismatch dir {h.dir_name(i)}"


@pytest.mark.parametrize("shape", [(20, 12, 9, 2), (64, 64, 64, 3)])
@pytest.mark.parametrize("remap", [0, 1, 2])
@pytest.mark.parametrize("order", ["xyzq", "qxyz"])
def test_box_move_matches_torch(tz, gpu, order, remap, shape):
    """direct transfer kernel: interior slab facing d -> ghost on side -d, all 26 at once, under
    each block order (0 round-robin, 1 and 2 the XCD-aware orders with padded launches). The
    64^3 grid gives faces of 9-18 blocks (more than 8 and not a multiple of 8), so the per-box
    remap's reordering and its grid-stride loop over the real blocks run, not only the padding"""
    a = tz.HaloArgs()
    a.nx, a.ny, a.nz, a.ghost = shape
    a.nq = 3
    a.neighbors, a.order = 26, order
    h = tz.HaloExchange(a)
    grid = torch.randn(h.grid_elems(), dtype=torch.float64, device="cuda")
    out = grid.clone()
    exp = grid.clone()
    moves = []
    for i in range(h.ndirs()):
        s, d = h.pack_box(i), h.unpack_box(h.opposite(i))
        moves.append(dict(src=out.data_ptr(), dst=out.data_ptr(), src_off=s["grid_off"],
                          dst_off=d["grid_off"], s1=s["s1"], s2=s["s2"], s3=s["s3"],
                          len=s["len"], n1=s["n1"], n2=s["n2"], n3=s["n3"]))
        for i3 in range(s["n3"]):
            for i2 in range(s["n2"]):
                so = s["grid_off"] + i2 * s["s2"] + i3 * s["s3"]
                do = d["grid_off"] + i2 * s["s2"] + i3 * s["s3"]
                exp.as_strided((s["n1"], s["len"]), (s["s1"], 1), do).copy_(
                    grid.as_strided((s["n1"], s["len"]), (s["s1"], 1), so))
    prev = tz._tz.kernels.get_xcd_remap()
    tz._tz.kernels.set_xcd_remap(remap)
    try:
        tz._tz.kernels.box_move_many(moves, _stream())
        torch.cuda.synchronize()
    finally:
        tz._tz.kernels.set_xcd_remap(prev)
    assert torch.equal(out, exp)


def test_box_copy_many_equals_single(tz, gpu):
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = 16
    a.neighbors = 26
    h = tz.HaloExchange(a)
    grid = torch.randn(h.grid_elems(), dtype=torch.float64, device="cuda")
    boxes, bufs1, bufs2 = [], [], []
    for i in range(h.ndirs()):
        b = h.pack_box(i)
        cnt = b["len"] * b["n1"] * b["n2"] * b["n3"]
        t1 = torch.zeros(cnt, dtype=torch.float64, device="cuda")
        t2 = torch.zeros(cnt, dtype=torch.float64, device="cuda")
        b1 = dict(b, buf=t1.data_ptr())
        tz._tz.kernels.box_copy(grid.data_ptr(), b1, False, _stream())
        boxes.append(dict(b, buf=t2.data_ptr()))
        bufs1.append(t1)
        bufs2.append(t2)
    tz._tz.kernels.box_copy_many(grid.data_ptr(), boxes, False, _stream())
    torch.cuda.synchronize()
    for t1, t2 in zip(bufs1, bufs2):
        assert torch.equal(t1, t2)


@pytest.mark.parametrize("lanes,per_row", [(0, 10), (1, 10), (4, 10), (8, 10), (16, 10),
                                           (64, 10), (-1, 10), (-1, 90), (16, 90),
                                           (1001, 10), (1002, 10), (1004, 10), (1001, 40),
                                           (1004, 90)])
def test_csr_spmv_matches_torch(tz, gpu, lanes, per_row):
    # per_row 90: a 64-row CSR-stream block holds > 4096 nnz, exercising its multi-pass path;
    # 1000 + W: the ILP kernel (16 entries per lane group and pass: 40 / 90 take several passes)
    n = 5000
    rp, ci, val = tz._tz.random_band_matrix(n, 300, per_row * n, 7)
    rp_t = torch.tensor(rp, dtype=torch.int32, device="cuda")
    ci_t = torch.tensor(ci, dtype=torch.int32, device="cuda")
    v_t = torch.tensor(val, dtype=torch.float32, device="cuda")
    x = torch.randn(n, dtype=torch.float32, device="cuda")
    y = torch.zeros(n, dtype=torch.float32, device="cuda")
    tz._tz.kernels.csr_spmv(n, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(),
                            y.data_ptr(), lanes, False, _stream())
    A = torch.sparse_csr_tensor(rp_t.long().cpu(), ci_t.long().cpu(), v_t.cpu(), size=(n, n)).to_dense()
    ref = A.double() @ x.double().cpu()
    torch.cuda.synchronize()
    assert torch.allclose(y.double().cpu(), ref, rtol=1e-4, atol=1e-4)
    # accumulate variant
    tz._tz.kernels.csr_spmv(n, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(),
                            y.data_ptr(), lanes, True, _stream())
    torch.cuda.synchronize()
    assert torch.allclose(y.double().cpu(), 2 * ref, rtol=1e-4, atol=2e-4)


def test_vector_kernels(tz, gpu):
    n = 100_003
    a = torch.randn(n, device="cuda")
    b = torch.randn(n, device="cuda")
    y = torch.empty(n, device="cuda")
    tz._tz.kernels.vector_add_f32(n, a.data_ptr(), b.data_ptr(), y.data_ptr(), _stream())
    idx = torch.randint(0, n, (777,), dtype=torch.int32, device="cuda")
    g = torch.empty(777, device="cuda")
    tz._tz.kernels.gather_f32(777, a.data_ptr(), idx.data_ptr(), g.data_ptr(), _stream())
    xd = torch.randn(n, dtype=torch.float64, device="cuda")
    yd = torch.randn(n, dtype=torch.float64, device="cuda")
    yd0 = yd.clone()
    tz._tz.kernels.axpy_f64(n, 2.5, xd.data_ptr(), yd.data_ptr(), _stream())
    io = torch.empty(1000, dtype=torch.float64, device="cuda")
    tz._tz.kernels.iota_f64(1000, 3.0, 0.5, io.data_ptr(), _stream())
    torch.cuda.synchronize()
    assert torch.equal(y, a + b)
    assert torch.equal(g, a[idx.long()])
    assert torch.allclose(yd, yd0 + 2.5 * xd)
    assert torch.equal(io, 3.0 + 0.5 * torch.arange(1000, dtype=torch.float64, device="cuda"))


@pytest.fixture(params=[(16, 16, 1, 0), (16, 64, 1, 0), (8, 32, 2, 0), (16, 16, 2, 0), (16, 16, 1, 1),
                        (8, 64, 1, 1)], ids=lambda t: "ty%d-zc%d-pf%d-xcd%d" % t)
def stencil_tuning(tz, request):
    """kernel tilings (rows per tile, planes per chunk, planes in flight, XCD-contiguous tile
    order); restores the default"""
    prev = tz._tz.kernels.get_stencil_xcd_tiles()
    tz._tz.kernels.set_stencil_tuning(*request.param[:3])
    tz._tz.kernels.set_stencil_xcd_tiles(bool(request.param[3]))
    yield request.param
    tz._tz.kernels.set_stencil_tuning()
    tz._tz.kernels.set_stencil_xcd_tiles(prev)


@pytest.mark.parametrize("nx", [100, 99, 1])  # even rows: 2 per thread; odd: 1; 1: thin box
@pytest.mark.parametrize("lds", [True, False])
@pytest.mark.parametrize("order", ["qxyz", "xyzq"])
def test_stencil7_matches_torch(tz, gpu, order, lds, nx, stencil_tuning):
    """7-point stencil over a box with a one-cell apron, both storage orders, box extents that
    are not multiples of the tile (64 x 8 x 32 planes), against a torch fp64 reference"""
    torch = pytest.importorskip("torch")
    nq, ny, nz, pad = 3, 37, 45, 5
    c0, c1 = 0.4, 0.1
    if order == "qxyz":
        P = nq * (nx + 2 + 2 * pad)
        G = torch.randn(nz + 2, ny + 2, P, dtype=torch.float64, device="cuda")
        O = torch.zeros_like(G)
        x0 = nq * (1 + pad)  # first box element in a row
        row, xs, sy, sz, so, nouter = nq * nx, nq, P, P * (ny + 2), 0, 1
        base = sz + sy + x0

        def sl(t, dz, dy, dx):
            return t[1 + dz:nz + 1 + dz, 1 + dy:ny + 1 + dy, x0 + dx:x0 + dx + row]
    else:
        P = nx + 2 + 2 * pad
        G = torch.randn(nq, nz + 2, ny + 2, P, dtype=torch.float64, device="cuda")
        O = torch.zeros_like(G)
        x0 = 1 + pad
        row, xs, sy, sz, nouter = nx, 1, P, P * (ny + 2), nq
        so = sz * (nz + 2)
        base = sz + sy + x0

        def sl(t, dz, dy, dx):
            return t[:, 1 + dz:nz + 1 + dz, 1 + dy:ny + 1 + dy, x0 + dx:x0 + dx + row]
    tz._tz.kernels.stencil7(G.data_ptr(), O.data_ptr(), base, row, ny, nz, nouter, sy, sz, so, xs,
                            c0, c1, lds, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = c0 * sl(G, 0, 0, 0) + c1 * (sl(G, 0, 0, -xs) + sl(G, 0, 0, xs) + sl(G, 0, -1, 0) +
                                      sl(G, 0, 1, 0) + sl(G, -1, 0, 0) + sl(G, 1, 0, 0))
    got = sl(O, 0, 0, 0)
    assert torch.allclose(got, ref, rtol=1e-13, atol=1e-13), (got - ref).abs().max()
    # nothing outside the box is written
    assert float(O.abs().sum()) == pytest.approx(float(got.abs().sum()), rel=1e-12)


@pytest.mark.parametrize("ntload,ntstore", [(False, False), (False, True), (True, False), (True, True)])
def test_box_move_cache_policies(tz, gpu, ntload, ntstore):
    """every load / store cache policy of the move kernel moves the same data"""
    a = tz.HaloArgs()
    a.nx, a.ny, a.nz, a.ghost, a.nq = 64, 40, 24, 3, 3
    a.neighbors, a.order = 26, "qxyz"
    h = tz.HaloExchange(a)
    grid = torch.randn(h.grid_elems(), dtype=torch.float64, device="cuda")
    out, exp = grid.clone(), grid.clone()
    moves = []
    for i in range(h.ndirs()):
        s, d = h.pack_box(i), h.unpack_box(h.opposite(i))
        moves.append(dict(src=out.data_ptr(), dst=out.data_ptr(), src_off=s["grid_off"],
                          dst_off=d["grid_off"], s1=s["s1"], s2=s["s2"], s3=s["s3"],
                          len=s["len"], n1=s["n1"], n2=s["n2"], n3=s["n3"]))
        for i3 in range(s["n3"]):
            for i2 in range(s["n2"]):
                so = s["grid_off"] + i2 * s["s2"] + i3 * s["s3"]
                do = d["grid_off"] + i2 * s["s2"] + i3 * s["s3"]
                exp.as_strided((s["n1"], s["len"]), (s["s1"], 1), do).copy_(
                    grid.as_strided((s["n1"], s["len"]), (s["s1"], 1), so))
    k = tz._tz.kernels
    prev, prev_st = k.get_box_tuning(), k.get_nt_move_store()
    try:
        k.set_box_tuning(prev[0], prev[1], prev[2], prev[3], ntload)
        k.set_nt_move_store(ntstore)
        k.box_move_many(moves, _stream())
        torch.cuda.synchronize()
    finally:
        k.set_box_tuning(*prev)
        k.set_nt_move_store(prev_st)
    assert torch.equal(out, exp)


def _rows(box, lead=0, trail=0):
    """(offset, length) of every grid row of a box, widened by lead / trail elements"""
    for i3 in range(box["n3"]):
        for i2 in range(box["n2"]):
            for i1 in range(box["n1"]):
                yield (box["grid_off"] + i1 * box["s1"] + i2 * box["s2"] + i3 * box["s3"] - lead,
                       lead + box["len"] + trail)


def _mask(n, boxes, widened):
    m = torch.zeros(n, dtype=torch.bool)
    for b in boxes:
        for off, ln in _rows(b, *((b["lead"], b["trail"]) if widened else (0, 0))):
            m[off:off + ln] = True
    return m.to("cuda")


@pytest.mark.parametrize("align", [16, 8])
@pytest.mark.parametrize("order", ["xyzq", "qxyz"])
@pytest.mark.parametrize("neighbors", [6, 26])
def test_widened_unpack_matches_torch(tz, gpu, order, neighbors, align):
    """the unpack through unpack_box(i), whose x-ghost rows are widened over
    the row padding (lead / trail > 0), from a random buffer, one box at a time and all boxes in
    one batch. Every logical ghost cell is exact (torch strided reference), nothing outside
    [row start - lead, row end + trail) changes, and the widened elements are padding: no pack
    or unpack box of any direction covers them."""
    a = tz.HaloArgs()
    a.nx, a.ny, a.nz, a.nq, a.ghost = 20, 12, 9, 3, 3
    a.neighbors, a.order, a.ghost_align = neighbors, order, align
    h = tz.HaloExchange(a)
    n = h.grid_elems()
    grid = torch.randn(n, dtype=torch.float64, device="cuda")
    ub = [h.unpack_box(i) for i in range(h.ndirs())]
    pb = [h.pack_box(i) for i in range(h.ndirs())]
    assert any(b["lead"] > 0 or b["trail"] > 0 for b in ub), "no widened box: the test is void"
    logical_all = _mask(n, ub + pb, False)
    srcs, exp_all = [], grid.clone()
    for i, b in enumerate(ub):
        cnt = b["len"] * b["n1"] * b["n2"] * b["n3"]
        src = torch.randn(cnt, dtype=torch.float64, device="cuda")
        srcs.append(src)
        b["buf"] = src.data_ptr()
        # one box: exact ghost cells, changes only inside the widened rows
        g2 = grid.clone()
        tz._tz.kernels.box_copy(g2.data_ptr(), b, True, _stream())
        exp = grid.clone()
        srcv = src.view(b["n3"], b["n2"], b["n1"], b["len"])
        for i3 in range(b["n3"]):
            for i2 in range(b["n2"]):
                base = b["grid_off"] + i2 * b["s2"] + i3 * b["s3"]
                for e in (exp, exp_all):
                    e.as_strided((b["n1"], b["len"]), (b["s1"], 1), base).copy_(srcv[i3, i2])
        torch.cuda.synchronize()
        mine, allowed = _mask(n, [b], False), _mask(n, [b], True)
        assert torch.equal(g2[mine], exp[mine]), f"ghost cells wrong, box {h.dir_name(i)}"
        assert torch.equal(g2[~allowed], grid[~allowed]), "unpack wrote outside its widened rows"
        # the widening covers row padding only
        assert not (allowed & ~mine & logical_all).any(), "widened over a logical cell"
    # all boxes in one batch launch
    g3 = grid.clone()
    tz._tz.kernels.box_copy_many(g3.data_ptr(), ub, True, _stream())
    torch.cuda.synchronize()
    allowed = _mask(n, ub, True)
    ghosts = _mask(n, ub, False)
    assert torch.equal(g3[ghosts], exp_all[ghosts])
    assert torch.equal(g3[~allowed], grid[~allowed])


@pytest.mark.parametrize("lanes", [1004, 1002, 1001])
@pytest.mark.parametrize("order", ["qxyz", "xyzq"])
def test_box_move_spmv_matches_torch(tz, gpu, order, lanes):
    """horizontal fusion: the 26-direction move and a CSR SpMV in one launch (their workgroups
    interleaved) give exactly the move's ghosts (torch strided copy) and the SpMV's y (torch
    fp64 product), with rows that need several passes of the ILP kernel; then accumulate"""
    a = tz.HaloArgs()
    a.nx, a.ny, a.nz, a.ghost, a.nq = 40, 24, 18, 3, 3
    a.neighbors, a.order = 26, order
    h = tz.HaloExchange(a)
    grid = torch.randn(h.grid_elems(), dtype=torch.float64, device="cuda")
    out, exp = grid.clone(), grid.clone()
    moves = []
    for i in range(h.ndirs()):
        s, d = h.pack_box(i), h.unpack_box(h.opposite(i))
        moves.append(dict(src=out.data_ptr(), dst=out.data_ptr(), src_off=s["grid_off"],
                          dst_off=d["grid_off"], s1=s["s1"], s2=s["s2"], s3=s["s3"],
                          len=s["len"], n1=s["n1"], n2=s["n2"], n3=s["n3"]))
        for i3 in range(s["n3"]):
            for i2 in range(s["n2"]):
                so = s["grid_off"] + i2 * s["s2"] + i3 * s["s3"]
                do = d["grid_off"] + i2 * s["s2"] + i3 * s["s3"]
                exp.as_strided((s["n1"], s["len"]), (s["s1"], 1), do).copy_(
                    grid.as_strided((s["n1"], s["len"]), (s["s1"], 1), so))
    n = 30_000
    rp, ci, val = tz._tz.random_band_matrix(n, 500, 40 * n, 11)  # 40 per row: several passes
    rp_t = torch.tensor(rp, dtype=torch.int32, device="cuda")
    ci_t = torch.tensor(ci, dtype=torch.int32, device="cuda")
    v_t = torch.tensor(val, dtype=torch.float32, device="cuda")
    x = torch.randn(n, dtype=torch.float32, device="cuda")
    y = torch.full((n,), 7.0, dtype=torch.float32, device="cuda")
    A = torch.sparse_csr_tensor(rp_t.long().cpu(), ci_t.long().cpu(), v_t.cpu(), size=(n, n)).to_dense()
    ref = A.double() @ x.double().cpu()
    args = (n, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(), x.data_ptr(), y.data_ptr(), lanes)
    tz._tz.kernels.box_move_spmv(moves, *args, False, _stream())
    torch.cuda.synchronize()
    assert torch.equal(out, exp)
    assert torch.allclose(y.double().cpu(), ref, rtol=1e-4, atol=1e-4)
    tz._tz.kernels.box_move_spmv(moves, *args, True, _stream())  # y += A x; the move again
    torch.cuda.synchronize()
    assert torch.equal(out, exp)
    assert torch.allclose(y.double().cpu(), 2 * ref, rtol=1e-4, atol=2e-4)
    # SpMV only / move only: the same launcher with an empty half
    y.zero_()
    tz._tz.kernels.box_move_spmv([], *args, False, _stream())
    out2 = grid.clone()
    for m in moves:
        m["src"] = m["dst"] = out2.data_ptr()
    tz._tz.kernels.box_move_spmv(moves, 0, 0, 0, 0, 0, 0, lanes, False, _stream())
    torch.cuda.synchronize()
    assert torch.allclose(y.double().cpu(), ref, rtol=1e-4, atol=1e-4)
    assert torch.equal(out2, exp)


@pytest.mark.parametrize("nx,g", [(24, 3), (16, 4), (20, 3)])
def test_row_pair_moves_match_torch(tz, gpu, nx, g):
    """the x self-wrap of the reference's XYZQ layout (x = 0 at the row start) as one row pair
    against the two plain moves in torch; the whole grid is compared"""
    from test_move_kinds import _pair_moves

    h, m = _pair_moves(tz, nx, g, base=1)  # geometry only; pointers below
    grid = torch.randn(h.grid_elems(), dtype=torch.float64, device="cuda")
    out, exp = grid.clone(), grid.clone()
    m = dict(m, src=out.data_ptr(), dst=out.data_ptr())
    assert tz._tz.kernels.move_kinds([m]) == ["pair"]
    delta, L = m["dst_off"] - m["src_off"], m["len"]
    runs = [(m["src_off"], m["dst_off"]), (m["src_off"] + L + delta, m["src_off"] + L)]
    for i3 in range(m["n3"]):
        for i2 in range(m["n2"]):
            for so, do in runs:
                o = i2 * m["s2"] + i3 * m["s3"]
                exp.as_strided((m["n1"], L), (m["s1"], 1), do + o).copy_(
                    grid.as_strided((m["n1"], L), (m["s1"], 1), so + o))
    tz._tz.kernels.box_move_many([m], _stream())
    torch.cuda.synchronize()
    assert torch.equal(out, exp)
