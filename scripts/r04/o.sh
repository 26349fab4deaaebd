# r04 o: ablations of the deferred accounting (as its own kernel): which part holds its ~16 us
R=$(pwd)
O=$R/gpurun_out/r04o; mkdir -p $O
export PYTHONUNBUFFERED=1
for a in 0 1 2 4 7; do
  timeout -k 10 200 env NSGPU_P2P_SDEF_KERNEL=1 NSGPU_P2P_SDEF_ABL=$a python bench.py --no-cpu-baseline --no-secondary --steps 2 > $O/abl_$a.log 2>&1
  rc=$?; echo "abl $a rc=$rc" >> $O/rc.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
exit 0
