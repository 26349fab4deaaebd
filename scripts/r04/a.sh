# r04 a: graph side-branch probe + baseline default bench
set -e
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 60 ./scripts/build/probe_graph 8 12 > $O/probe_graph_8_12.log 2>&1
timeout -k 10 60 ./scripts/build/probe_graph 3 10 > $O/probe_graph_3_10.log 2>&1
timeout -k 10 60 ./scripts/build/probe_graph 1 10 > $O/probe_graph_1_10.log 2>&1
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mixed.py tests/test_gpu_plugin.py tests/test_gpu_wifi_dist.py > $O/pytest_mixed_plugin.log 2>&1
