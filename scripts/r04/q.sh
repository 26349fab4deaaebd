# r04 q: per-block times of k2_pa / k2_handle in the deferred pipeline (diagnostic build)
R=$(pwd)
O=$R/gpurun_out/r04q; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/r04/blocks_df.py > $O/blocks.log 2>&1
echo "rc=$?" >> $O/rc.log
exit 0
