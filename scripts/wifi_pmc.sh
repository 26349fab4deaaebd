set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc/kt -o run -- python3 $R/scripts/wifi_once.py 0.5 > $R/gpurun_out/pmc/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_BRANCH -d $R/gpurun_out/pmc/p1 -o run -- python3 $R/scripts/wifi_once.py 0.5 > $R/gpurun_out/pmc/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR -d $R/gpurun_out/pmc/p2 -o run -- python3 $R/scripts/wifi_once.py 0.5 > $R/gpurun_out/pmc/p2.log 2>&1
