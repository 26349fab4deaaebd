# r04 l: where k2_rank's time goes — the deferred accounting as its own kernel (k2_rank = bookkeeping +
# tiles; k2_sdef alone), eager profile of the bench line
R=$(pwd)
O=$R/gpurun_out/r04l; mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/rc.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step bench_sdefk 300 env NSGPU_P2P_SDEF_KERNEL=1 python bench.py --no-cpu-baseline --no-secondary
step bench_nodefer 300 env NSGPU_P2P_NODEFER=1 python bench.py --no-cpu-baseline --no-secondary
exit 0
