"""The RCCL self-exchange test (tests/test_gpu_runtime.py::test_halo_rccl_self_exchange) as a
plain script, so it can run without torch (TZ_NO_TORCH=1: the system ROCm runtime)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import tenzing_amd as tz
    from tenzing_amd.models import HaloConfig, build_halo
    from tenzing_amd.utils.env import runtime_libraries

    print(runtime_libraries(), flush=True)
    halo, g = build_halo(HaloConfig(n=24, neighbors=6, transport="rccl"), tz.SelfCtrl(), device=0)
    print("built; transports", halo.transport_report(), flush=True)
    for m in (tz.ExecMode.Eager, tz.ExecMode.Graph):
        rt = tz.HipRuntime(device=0, n_streams=2, mode=m, graph_unroll=3)
        for seed in (4, 5):
            seq = tz.random_rollout(tz.State(g, tz.Platform(2)), seed)
            halo.init_grid()
            rt.prepare(seq)
            print(m, seed, "prepared", rt.effective_mode, rt.graph_nodes(), flush=True)
            rt.run(1)
            rt.device_sync()
            b1 = halo.check_grid()
            rt.run(7)
            rt.device_sync()
            print(m, seed, "bad", b1, halo.check_grid(), flush=True)


if __name__ == "__main__":
    main()
