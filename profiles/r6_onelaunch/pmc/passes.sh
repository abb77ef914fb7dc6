set -o pipefail
P="python3 scripts/coexec_probe.py --iters 2 --reps 2 --lanes 1004"
mkdir -p gpurun_out/pmc_ol
i=0
for c in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_ol/p$i -o run -- $P > gpurun_out/pmc_ol/p$i.log 2>&1 || exit $?
done
