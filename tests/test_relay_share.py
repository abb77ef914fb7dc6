"""Relay share from the link model: on the 2x2x2 grid every idle-link path
to a face peer runs through the corner peer, so the relayed bytes of all 6 faces share one
link; f* = r_corner / (r_corner + 3 r_face) balances it against the face links (0.25 at equal
rates). Checked on the bytes the halo ops themselves report (GpuOp.traffic, the simulator's
input), rank 0 of 8, no GPU."""
import pytest

from tenzing_amd.parallel.linkmodel import (relay_fracs_offered, relay_share,
                                            relay_share_from_record)


def test_f_star_formula():
    assert relay_share() == pytest.approx(0.25)
    # a slower corner link takes a smaller share, a faster one more
    assert relay_share(60.0, 30.0) == pytest.approx(30 / 210)
    assert relay_share(60.0, 120.0) == pytest.approx(120 / 300)
    assert relay_fracs_offered(0.25) == (0.15, 0.2, 0.25)
    assert relay_fracs_offered(0.9) == (0.15, 0.2, 0.45)
    with pytest.raises(ValueError):
        relay_share(0.0, 1.0)


def test_f_star_from_a_records_link_matrix():
    row = [-1, 70.0, 70.0, 50.0, 70.0, 50.0, 50.0, 35.0]
    rec = {"config": {"rank_grid": [2, 2, 2]}, "link_matrix": {"why": "", "put_GBps": [row]}}
    assert relay_share_from_record(rec) == pytest.approx(35 / (35 + 210))
    assert relay_share_from_record({"config": {"rank_grid": [1, 2, 4]}}) is None


def _link_bytes(seq):
    per = {}
    for o in seq.ops():
        for res, _eng, b in o.traffic():
            if res.startswith("xgmi"):
                per[res] = per.get(res, 0.0) + b
    return per


def test_busiest_link_with_f_star_on_the_2x2x2_model(monkeypatch):
    monkeypatch.setenv("TZ_IPC_GRID", "0")  # receive buffers: the relay is offered
    import tenzing_amd as tz
    from tenzing_amd.parallel.linkmodel import headline_graph, transport_seeds

    h, g = headline_graph(0, 8)
    assert tuple(h.rank_grid()) == (2, 2, 2)
    seeds, alts = transport_seeds(g, tz.Platform(4), 4)
    by = {a: s for a, s in zip(alts, seeds)}
    put = next(s for a, s in by.items() if a == "he_via_ipc")
    base = _link_bytes(put)
    pair = max(base.values())  # both faces of an axis over one link
    f_star = relay_share()
    rl = [s for a, s in by.items() if a == f"he_via_relay{round(f_star * 100)}"]
    assert rl, list(by)
    for s in rl:
        links = _link_bytes(s)
        busiest = max(links.values())
        assert busiest <= 0.76 * pair, (busiest / pair, links)
        # the corner link carries the 6 relayed shares, about as much as each face link
        corner = links["xgmi:7"]
        face = max(links[f"xgmi:{q}"] for q in (1, 2, 4))
        assert corner == pytest.approx(face, rel=0.05), links
    # the fixed 0.2 share leaves the face links busier
    rl20 = [s for a, s in by.items() if a == "he_via_relay20"]
    assert max(max(_link_bytes(s).values()) for s in rl20) > 0.79 * pair
