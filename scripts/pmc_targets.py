#!/usr/bin/env python3
"""Fixed set of kernel launches for rocprofv3 counter collection (--pmc): the halo direct move
(all 26 directions), fused pack / unpack, the SpMV kernels and rocSPARSE's CSR SpMV, each a
few times.

  rocprofv3 --pmc FETCH_SIZE --output-format csv -d out -- python3 scripts/pmc_targets.py
  rocprofv3 --pmc WRITE_SIZE ... -- python3 scripts/pmc_targets.py --only-move 20   # headline only
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tenzing_amd as tz  # noqa: E402
from tenzing_amd.models import HaloConfig, build_halo  # noqa: E402


def main():
    torch.zeros(1, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    order = os.environ.get("TZ_PMC_ORDER", "qxyz")  # xyzq: the reference driver's layout
    # ghost alignment (-1: x = 0 at the row start, the reference's) and extra row pitch
    align = int(os.environ.get("TZ_PMC_ALIGN", "16"))
    pad = int(os.environ.get("TZ_PMC_PITCH_PAD", "0"))
    hd, _ = build_halo(HaloConfig(n=512, neighbors=26, order=order, transport="direct",
                                  ghost_align=align, pitch_pad=pad),
                       tz.SelfCtrl(), device=0)
    if len(sys.argv) > 2 and sys.argv[1] == "--only-move":
        # steady state of the headline: the 26-direction move back to back, as in the hipGraph
        # loop (the caches hold what the previous exchange left)
        alld = list(range(hd.ndirs()))
        for _ in range(int(sys.argv[2])):
            hd.direct_group(alld, st)
        torch.cuda.synchronize()
        return
    hc, _ = build_halo(HaloConfig(n=512, neighbors=26, order="qxyz", transport="copy"),
                       tz.SelfCtrl(), device=0)
    alld = list(range(hd.ndirs()))
    for _ in range(3):
        hd.direct_group(alld, st)
        hc.pack_all(st)
        hc.shift_all(st)
        hc.unpack_all(st)
    hs, _ = build_halo(HaloConfig(n=512, neighbors=26, order="qxyz", transport="direct",
                                  stencil=True), tz.SelfCtrl(), device=0)
    for _ in range(3):
        hs.stencil(2, st)  # whole interior: 2.5-D LDS-tiled 7-point stencil
        hs.stencil(1, st)  # the one-cell shell (thin-slab kernel)
    del hs
    torch.cuda.synchronize()
    m = 150_000
    rp, ci, val = tz._tz.random_band_matrix(m, m, 10 * m, 1)
    rp_t = torch.tensor(rp, dtype=torch.int32, device="cuda")
    ci_t = torch.tensor(ci, dtype=torch.int32, device="cuda")
    v_t = torch.tensor(val, dtype=torch.float32, device="cuda")
    x = torch.randn(m, device="cuda")
    y = torch.zeros(m, device="cuda")
    lib = tz._tz.kernels.RocsparseCsr(m, m, ci_t.numel(), rp_t.data_ptr(), ci_t.data_ptr(),
                                      v_t.data_ptr(), x.data_ptr(), y.data_ptr(), "adaptive")
    for _ in range(3):
        for lanes in (8, -1):
            tz._tz.kernels.csr_spmv(m, rp_t.data_ptr(), ci_t.data_ptr(), v_t.data_ptr(),
                                    x.data_ptr(), y.data_ptr(), lanes, False, st)
        lib.run(st)  # rocSPARSE (library comparison)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
