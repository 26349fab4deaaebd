#!/bin/bash
# Round 3, session b: (1) the rocprofv3 SIGSEGV of round 2 — config 4 replayed from its hipGraph under
# --kernel-trace with a symbolizing SIGSEGV handler (scripts/segv_dump.so); (2) per-block window timing
# at HEAD (diagnostic build).  Each GPU step has its own limit; a fault ends the script.
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/graph_trace -o run \
    -- python3 scripts/rocprof_graph_probe.py 2 > $O/rocprof_graph_probe.log 2>&1
rc=$?
echo "rocprof_graph_probe rc=$rc" | tee $O/steps.log
tail -60 $O/rocprof_graph_probe.log | cut -c1-300
rocprofv3 --version > $O/rocprofv3_version.txt 2>&1 || true
if [ $rc -ne 0 ] && [ $rc -ne 139 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ $rc -eq 139 ]; then exit 0; fi
timeout -k 10 200 python3 scripts/p2p_blocks.py 128 > $O/blocks.log 2>&1
echo "blocks rc=$?" | tee -a $O/steps.log
cat $O/blocks.log | head -60
