"""Host-side checks of the RCCL communication ops (no GPU needed); the ops themselves run in
tests/test_gpu_comm_ops.py."""
import pytest


def test_comm_op_classes_exported(tz):
    for name in ("CommOp", "SendRecvOp", "AlltoallvOp", "AllReduceOp", "AllGatherOp",
                 "ReduceScatterOp", "BroadcastOp"):
        assert hasattr(tz, name), name
    assert issubclass(tz.SendRecvOp, tz.CommOp)
    assert tz.RcclComm.dtype_size(4) == 2 and tz.RcclComm.dtype_size(1) == 8
    with pytest.raises(tz.TzError):
        tz.RcclComm.dtype_size(9)


def test_comm_ops_need_communicators(tz):
    with pytest.raises(tz.TzError, match="communicator"):
        tz.SendRecvOp("sr", [], 0, 0, 0, 0, 0, 0, 1)
    with pytest.raises(tz.TzError, match="communicator"):
        tz.AllReduceOp("ar", [], 0, 0, 0, 1)


def test_torch_front_end_checks(tz):
    torch = pytest.importorskip("torch")
    from tenzing_amd.ops import comm

    cpu = torch.zeros(4)
    with pytest.raises(ValueError, match="GPU"):
        comm.all_reduce("ar", [object()], cpu)
    with pytest.raises(ValueError, match="communicator"):
        comm._comms([])
    with pytest.raises(ValueError, match="reduction"):
        comm._red("mean")
    with pytest.raises(ValueError):
        comm.send_recv("sr", [object()], None, 0, None, 0)
    assert comm.DTYPES[torch.bfloat16] == 4 and comm.REDUCTIONS["max"] == 2
