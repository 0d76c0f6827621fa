# DAG traces of the default library and variant builds: continuation/drawn POTRF phases
mkdir -p gpurun_out
for v in default "$@"; do
  if [ $v = default ]; then lib=ar_slam_amd/libarslam_lm.so; else lib=ar_slam_amd/var_$v.so; fi
  ARSLAM_LIB=$PWD/$lib ARSLAM_DAG_TRACE=gpurun_out/dag_$v.bin ARSLAM_DAG_TRACE_SKIP=3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-incremental --steps 1 --warmup 1 > gpurun_out/tr_$v.log 2>&1 || { tail gpurun_out/tr_$v.log; exit 1; }
  echo "== $v"; python tools/potrf_cont.py gpurun_out/dag_$v.bin; python tools/dag_critical.py gpurun_out/dag_$v.bin | head -1
done
