#!/bin/bash
# Round 3 session p: wifi-grid phys-per-block sweep (fewer lanes per wave, more waves per SIMD), and the
# example's own Stop (32 s) as one bench step (reception table ~51 GB).
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
: > $O/sweep.log
for P in 0 3 4 5 6 8; do
  if [ "$P" = 0 ]; then unset NSGPU_WIFI_PHYS_PER_BLOCK; else export NSGPU_WIFI_PHYS_PER_BLOCK=$P; fi
  echo "P=$P" >> $O/sweep.log
  timeout -k 10 120 python -u bench.py --workload wifi-grid --steps 2 --warmup 1 --no-cpu-baseline > $O/one.log 2>&1
  rc=$?
  grep '^{' $O/one.log | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2), d['value'], d['roofline'].get('kernel_ms'))" >> $O/sweep.log
  if [ $rc -ne 0 ]; then echo "rc=$rc" >> $O/sweep.log; cat $O/sweep.log; exit $rc; fi
done
unset NSGPU_WIFI_PHYS_PER_BLOCK
cat $O/sweep.log
timeout -k 10 300 python -u bench.py --workload wifi-grid --wifi-stop 32 --steps 1 --warmup 0 --no-cpu-baseline > $O/stop32.log 2>&1
echo "stop32 rc=$?"
tail -1 $O/stop32.log | cut -c1-1200
