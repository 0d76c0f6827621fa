# diag16 / POTRF micro-benchmarks of variant builds tools/{diag16,potrf2}_bench_<V> (debug)
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  echo "== $v"; timeout -k 10 60 ./tools/diag16_bench_$v && timeout -k 10 60 ./tools/potrf2_bench_$v || exit 1
done
