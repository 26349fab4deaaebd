#!/bin/bash
# GPU-box runner for every measurement and test stage (one gpurun call: `bash scripts/measure_all.sh OUT STAGE...`).
# OUT is a directory name under gpurun_out/; each STAGE runs under its own time limit and the first failure ends
# the script (no GPU step runs after a failed one).  Stages:
#   tests            the whole -m gpu suite (one pytest process)
#   tests:<expr>     the -m gpu tests selected by -k <expr>
#   smoke            __graft_entry__.smoke ()
#   bench            the default bench line (config 4, driver-style)
#   benches          every workload's bench line (p2p grid, dumbbell, partitioned grid / dumbbell, wifi-loop, churn)
#   bench:<args>     one bench line with extra arguments (commas for spaces: bench:--workload,dumbbell)
#   rocprof_p2p      rocprofv3 kernel stats of the default bench (eager launches: the tracer cannot follow graphs)
#   rocprof_wifil    rocprofv3 kernel stats of the closed-loop Wi-Fi line
#   rocprof_dumbbell rocprofv3 kernel stats of the partitioned dumbbell line
#   rocprof_dumbbell1 rocprofv3 kernel trace + stats of the single engine's dumbbell line
#   rocprof_grid_part rocprofv3 kernel stats of the partitioned grid line (one rank)
#   pmc_p2p          config-4 HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes -> traffic_p2p-grid.json
#   pmc_lines        config-4 L2 / L1 request counters (TCC hit / miss / requests, TCP requests) per kernel
#   pmc_sq_part      wave-state counters (SQ busy / wait / VALU / LDS) of the partitioned grid's kernels
#   pmc_sq_p2p       wave-state counters (SQ wait / active / VMEM instructions) of config 4's kernels
#   py:<script>      python scripts/<script> (diagnostics), output to OUT/<script>.log
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$1
shift
mkdir -p $O
cd $R
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  echo "[$(date +%T)] $name" >> $O/steps.log
  if ! timeout -k 10 $secs "$@" > $O/$name.log 2>&1; then
    echo "[$(date +%T)] $name FAILED (rc $?)" >> $O/steps.log
    tail -30 $O/$name.log
    exit 1
  fi
}
for st in "$@"; do
  case $st in
    tests) step tests 1500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    tests:*) step tests_k 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "${st#tests:}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) step bench 300 python bench.py ;;
    bench:*) a=${st#bench:}; step bench_$(echo $a | tr -c 'a-zA-Z0-9\n' '_') 300 python bench.py ${a//,/ } ;;
    benches)
      step bench_p2p_grid 300 python bench.py
      step bench_dumbbell 300 python bench.py --workload dumbbell
      step bench_dumbbell_partitioned 300 python bench.py --workload dumbbell --partitioned
      step bench_p2p_grid_partitioned 300 python bench.py --partitioned --no-cpu-baseline
      step bench_wifi_loop 300 python bench.py --workload wifi-loop
      step bench_churn 300 python bench.py --workload churn ;;
    rocprof_p2p)
      cd /tmp
      NSGPU_P2P_EAGER=1 step rocprof_p2p 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_p2p -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary
      cd $R ;;
    rocprof_wifil)
      cd /tmp
      step rocprof_wifil 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_wifil -o run --output-format csv -- python3 $R/bench.py --workload wifi-loop --steps 1 --warmup 0 --no-cpu-baseline
      cd $R ;;
    rocprof_grid_part)
      cd /tmp
      NSGPU_P2P_EAGER=1 step rocprof_grid_part 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_grid_part -o run --output-format csv -- python3 $R/bench.py --partitioned --steps 1 --warmup 0 --no-cpu-baseline
      cd $R ;;
    rocprof_dumbbell)
      cd /tmp
      NSGPU_P2P_EAGER=1 step rocprof_dumbbell 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_dumbbell -o run --output-format csv -- python3 $R/bench.py --workload dumbbell --partitioned --steps 1 --warmup 0 --no-cpu-baseline
      cd $R ;;
    rocprof_dumbbell1)  # the single engine's dumbbell: every dispatch (kernel_trace.csv) and the stats
      cd /tmp
      NSGPU_P2P_EAGER=1 step rocprof_dumbbell1 240 rocprofv3 --kernel-trace --stats -d $O/rocprof_dumbbell1 -o run --output-format csv -- python3 $R/bench.py --workload dumbbell --steps 1 --warmup 0 --no-cpu-baseline --no-secondary
      cd $R ;;
    pmc_p2p)
      cd /tmp
      NSGPU_P2P_EAGER=1 step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_grid -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary
      NSGPU_P2P_EAGER=1 step pmc_write 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_grid -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary
      cd $R
      python scripts/pmc_traffic.py $O/pmc_fetch_grid $O/pmc_write_grid $O/traffic_p2p-grid.json k2_pa k2_handle k2_rank > $O/traffic_grid.log 2>&1 ;;
    pmc_lines)
      cd /tmp
      NSGPU_P2P_EAGER=1 step pmc_tcc 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --output-format csv -d $O/pmc_tcc -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary
      NSGPU_P2P_EAGER=1 step pmc_tcp 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/pmc_tcp -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary
      cd $R ;;
    pmc_sq_part)  # wave-state counters of the partitioned grid's kernels (one pass: 8 SQ + 1 GRBM counters)
      cd /tmp
      rocprofv3 -L > $O/avail_counters.txt 2>&1 || true
      NSGPU_P2P_EAGER=1 step pmc_sq_part 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq_part -o pmc -- python3 $R/bench.py --partitioned --steps 1 --warmup 0 --no-cpu-baseline
      cd $R ;;
    pmc_sq_p2p)  # wave-state counters of config 4's kernels (eager launches; one pass: 8 SQ counters)
      cd /tmp
      rocprofv3 -L > $O/avail_counters.txt 2>&1 || true
      NSGPU_P2P_EAGER=1 step pmc_sq_p2p 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM --output-format csv -d $O/pmc_sq_p2p -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-secondary
      cd $R ;;
    py:*) s=${st#py:}; step ${s%%.py*} 600 python scripts/${s//,/ } ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "[$(date +%T)] done" >> $O/steps.log
