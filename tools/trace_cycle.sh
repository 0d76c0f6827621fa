mkdir -p gpurun_out
ARSLAM_DAG_TRACE=gpurun_out/dag.bin ARSLAM_DAG_TRACE_SKIP=3 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/tr.log 2>&1 || { tail gpurun_out/tr.log; exit 1; }
python tools/dag_critical.py gpurun_out/dag.bin
python tools/dag_trace.py gpurun_out/dag.bin > gpurun_out/dagtr.txt; head -14 gpurun_out/dagtr.txt
