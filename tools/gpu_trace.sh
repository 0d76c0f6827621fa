# cfg3 k_factor_dag task timeline at HEAD: the critical path and the POTRF phases (debug)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ARSLAM_DAG_TRACE=gpurun_out/trace_cfg3.bin ARSLAM_DAG_TRACE_SKIP=${SKIP:-2} timeout -k 10 300 python -u tools/trace_cfg3.py ${CFG:-cfg3} > gpurun_out/trace_run.txt 2>&1 && cat gpurun_out/trace_run.txt &&
python tools/dag_critical.py gpurun_out/trace_cfg3.bin > gpurun_out/critical.txt 2>&1; python tools/potrf_cont.py gpurun_out/trace_cfg3.bin > gpurun_out/potrf_cont.txt 2>&1; head -40 gpurun_out/critical.txt; head -12 gpurun_out/potrf_cont.txt
