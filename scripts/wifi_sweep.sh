# Wi-Fi per-phy kernel: GPU tests, then the wifi-grid bench at the default plan and a phys-per-block sweep
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wifi.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_wifi.log 2>&1
: > gpurun_out/sweep.log
for P in ${SWEEP:-0}; do
  if [ "$P" = 0 ]; then unset NSGPU_WIFI_PHYS_PER_BLOCK; else export NSGPU_WIFI_PHYS_PER_BLOCK=$P; fi
  echo "P=$P" >> gpurun_out/sweep.log
  timeout -k 10 120 python -u bench.py --workload wifi-grid --steps 2 --warmup 1 --no-cpu-baseline | grep '^{' >> gpurun_out/sweep.log
done
