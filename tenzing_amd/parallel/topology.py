"""Device-pair facts of a multi-rank run: which GPU each peer rank sits on, whether this rank's
GPU can reach it peer-to-peer, and on which device the peer memory this rank mapped over IPC
reports itself. On one GPU (loopback ranks) every peer is ``same_device``; on an 8-GPU node none
should be, and every pair should have peer access over xGMI. The record makes the first real
multi-GPU run explain itself: a transport that fails there can be matched to the pair it ran on.

Reference: the reference binds ``rank % cudaGetDeviceCount`` and never checks peers
(tenzing-mcts/examples/spmv_run_strategy.cuh:81-90); its data plane is CUDA-aware MPI.
"""
from __future__ import annotations

from typing import Callable, Iterable


def pair_facts(my_device: int, my_bus: str, peer_bus: str, device_by_bus: Callable[[str], int],
               can_access: Callable[[int, int], bool], mapped_on: int | None) -> dict:
    """Facts for one peer: pure function of the queries (testable without GPUs)."""
    same = bool(my_bus) and my_bus.lower() == (peer_bus or "").lower()
    visible = device_by_bus(peer_bus) if peer_bus else -1
    if same:
        access, why = None, "same device (loopback): no peer link involved"
    elif visible < 0:
        access, why = None, "peer GPU not visible to this process (device isolation)"
    else:
        access = bool(can_access(my_device, visible))
        why = "peer access over the device link" if access else "hipDeviceCanAccessPeer says no"
    f = {"bus": peer_bus, "same_device": same, "visible_as": visible, "can_access_peer": access,
         "reason": why}
    if mapped_on is not None:
        f["ipc_mapped_on_device"] = mapped_on
        # memory of a peer on another GPU must not report this rank's own device
        f["ipc_mapping_consistent"] = (mapped_on == my_device) == same if mapped_on >= 0 else None
    return f


def peer_device_facts(ctrl, device: int, peers: Iterable[int], *, bus_of=None, device_by_bus=None,
                      can_access=None, ipc_mapped: dict | None = None) -> dict:
    """Collective (every rank calls it): allgather each rank's PCI bus id, then the facts of this
    rank's peers. The query functions default to the native HIP ones."""
    from .. import _tz

    bus_of = bus_of or _tz.pci_bus_id
    device_by_bus = device_by_bus or _tz.device_by_pci_bus_id
    can_access = can_access or _tz.can_access_peer
    mine = bus_of(device) if device >= 0 else ""
    buses = [b.decode() for b in ctrl.allgather(mine)]
    ipc_mapped = ipc_mapped or {}
    facts = {}
    for q in sorted(set(int(p) for p in peers)):
        if q == ctrl.rank:
            continue
        facts[str(q)] = pair_facts(device, mine, buses[q], device_by_bus, can_access,
                                   ipc_mapped.get(q))
    return {"device": device, "bus": mine, "peers": facts, "summary": summarize(facts)}


def summarize(facts: dict) -> str:
    if not facts:
        return "no peers"
    n = len(facts)
    same = sum(1 for f in facts.values() if f["same_device"])
    if same == n:
        return f"all {n} peer(s) on this rank's own device (loopback)"
    ok = sum(1 for f in facts.values() if f["can_access_peer"])
    bad_map = sum(1 for f in facts.values() if f.get("ipc_mapping_consistent") is False)
    s = f"{n - same} of {n} peer(s) on other devices, {ok} with peer access"
    if bad_map:
        s += f"; {bad_map} IPC mapping(s) report an unexpected device"
    return s


def matrix_summary(m) -> dict | None:
    """Off-diagonal summary of a link matrix (``link_matrix``'s ``put_GBps`` / ``sdma_GBps``):
    how many ordered pairs were measured and how evenly they carry (``spread`` = max / min). On
    an 8-GPU node with one xGMI hop between every pair the spread stays near 1; a pair routed
    through another GPU, or a link shared with other traffic, stands out as the minimum."""
    vals = sorted(v for r, row in enumerate(m or []) for q, v in enumerate(row) if r != q and v > 0)
    if not vals:
        return None
    n = len(vals)
    med = vals[n // 2] if n % 2 else 0.5 * (vals[n // 2 - 1] + vals[n // 2])
    worst = min(((r, q) for r, row in enumerate(m) for q, v in enumerate(row) if r != q and v > 0),
                key=lambda rq: m[rq[0]][rq[1]])
    return {"pairs": n, "min": vals[0], "median": med, "max": vals[-1],
            "spread": vals[-1] / vals[0], "slowest_pair": list(worst)}
