"""How the direct-move kernel moves each box (kernels.move_kinds, host only): the x self-wrap of
the reference's XYZQ layout (x = 0 at the row start) as one row pair, odd-offset rows peeled."""


def _pair_moves(tz, nx, g, ghost_align=-1, base=1 << 20):
    """the +x / -x self-wrap of one (dy, dz) = (0, 0) as one row-pair move (geometry from a
    HaloExchange that is not set up; `base` stands in for the grid pointer)"""
    a = tz.HaloArgs()
    a.nx = a.ny = a.nz = nx
    a.nq, a.ghost, a.neighbors, a.order, a.ghost_align = 3, g, 26, "xyzq", ghost_align
    h = tz.HaloExchange(a)
    plus = next(i for i in range(h.ndirs()) if h.dir(i) == (1, 0, 0))
    s, d = h.pack_box(plus), h.unpack_box(h.opposite(plus))
    m = dict(src=base, dst=base, src_off=s["grid_off"], dst_off=d["grid_off"], s1=s["s1"],
             s2=s["s2"], s3=s["s3"], len=s["len"], n1=s["n1"], n2=s["n2"], n3=s["n3"], pair=True)
    return h, m


def test_kinds_of_the_row_start_layout(tz):
    h, m = _pair_moves(tz, 512, 3)
    plain = dict(m, pair=False)
    # the +x slab starts at x = 512 (16-B aligned), the -x slab at x = 3 (peeled)
    minus = next(i for i in range(h.ndirs()) if h.dir(i) == (-1, 0, 0))
    s, d = h.pack_box(minus), h.unpack_box(h.opposite(minus))
    peeled = dict(plain, src_off=s["grid_off"], dst_off=d["grid_off"])
    k = tz._tz.kernels
    assert k.move_kinds([m, plain, peeled]) == ["pair", "vec8", "peeled"]
    prev = k.get_peel_moves()
    k.set_peel_moves(False)
    try:
        assert k.move_kinds([peeled]) == ["vec8"]
    finally:
        k.set_peel_moves(prev)
