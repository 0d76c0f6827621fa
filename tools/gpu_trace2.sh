# cfg3 task timelines of the default library and a variant (debug): POTRF phases of the root chain
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
touch ar_slam_amd/*.so
for v in base "$@"; do
  if [ $v = base ]; then unset ARSLAM_LIB; else export ARSLAM_LIB=$PWD/ar_slam_amd/var_$v.so; fi
  ARSLAM_DAG_TRACE=gpurun_out/trace_$v.bin ARSLAM_DAG_TRACE_SKIP=2 timeout -k 10 300 python -u tools/trace_cfg3.py cfg3 > gpurun_out/trace_run_$v.txt 2>&1 || exit 1
  python tools/potrf_cont.py gpurun_out/trace_$v.bin > gpurun_out/potrf_cont_$v.txt 2>&1
  python tools/dag_critical.py gpurun_out/trace_$v.bin > gpurun_out/critical_$v.txt 2>&1
  echo "== $v"; head -3 gpurun_out/potrf_cont_$v.txt; head -2 gpurun_out/critical_$v.txt
done
