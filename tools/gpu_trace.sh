set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/diag16_bench > gpurun_out/diag16.txt 2>&1 && cat gpurun_out/diag16.txt &&
timeout -k 10 60 ./tools/potrf2_bench > gpurun_out/potrf2.txt 2>&1 && cat gpurun_out/potrf2.txt &&
timeout -k 10 60 ./tools/lat_bench > gpurun_out/lat.txt 2>&1 && cat gpurun_out/lat.txt &&
ARSLAM_DAG_TRACE=gpurun_out/trace_cfg3.bin ARSLAM_DAG_TRACE_SKIP=3 timeout -k 10 300 python -u tools/trace_cfg3.py cfg3 > gpurun_out/trace_run.txt 2>&1 && cat gpurun_out/trace_run.txt &&
python tools/dag_critical.py gpurun_out/trace_cfg3.bin > gpurun_out/critical.txt 2>&1; python tools/potrf_cont.py gpurun_out/trace_cfg3.bin > gpurun_out/potrf_cont.txt 2>&1; head -30 gpurun_out/critical.txt
