#!/bin/bash
# Round-6 profile set on the box (each GPU step under its own time limit,
# stopping at the first failure): the -m gpu suite, the default bench line
# (box fingerprint and library build included), rocprofv3 kernel stats of the
# cfg3 bench, the PMC HBM-byte passes (FETCH_SIZE, WRITE_SIZE) and the MFMA
# pass; bulky rocprof directories removed after their summaries.
# usage: bash tools/profile_round6.sh <tag> [skip-tests]
set -o pipefail
export TMPDIR=/tmp
t=${1:-r06}
mkdir -p gpurun_out
touch ar_slam_amd/*.so oracle/*.so
sha256sum ar_slam_amd/*.so > gpurun_out/libs_$t.txt
if [ "$2" != "skip-tests" ]; then bash tools/gpu_tests.sh gpu_tests_$t || exit 1; fi
timeout -k 10 400 python bench.py > gpurun_out/bench_$t.json 2> gpurun_out/bench_$t.err || { tail -30 gpurun_out/bench_$t.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_$t.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['setup_time_s'], d['incremental_cfg2']['wall_s'], d['localize_cfg5']['value'], d.get('box_fingerprint'), d['library'])" || exit 1
bash tools/prof_bench.sh $t --steps 10 --warmup 2 --no-fingerprint > gpurun_out/prof_${t}_summary.txt || exit 1
cp $(find gpurun_out/prof_$t -name "*kernel_stats.csv") gpurun_out/kernel_stats_$t.csv
python3 tools/kstats.py gpurun_out/kernel_stats_$t.csv > gpurun_out/kernel_stats_$t.txt
rm -rf gpurun_out/prof_$t
bash tools/pmc_bench.sh $t --steps 3 --warmup 1 --no-fingerprint || exit 1
rm -rf gpurun_out/pmc_${t}_FETCH_SIZE gpurun_out/pmc_${t}_WRITE_SIZE
python3 -c "import json; d=json.load(open('gpurun_out/pmc_$t.json')); print('dominant', d['dominant'], d['hbm_bytes_per_launch'])"
bash tools/pmc_mfma.sh $t --steps 3 --warmup 1 || exit 1
rm -rf gpurun_out/pmcmfma_$t
cat gpurun_out/pmc_mfma_$t.json
# cfg5: the k_localize VALU-instruction pass (bench.py reads profiles/pmc_localize.json)
bash tools/pmc_cfg5.sh || exit 1
cp gpurun_out/p5/pmc_localize.json gpurun_out/pmc_localize_$t.json
rm -rf gpurun_out/p5/pmc
cat gpurun_out/pmc_localize_$t.json
# the multi-rank path over a one-rank RCCL communicator (the RCCL calls on hardware)
timeout -k 10 300 python bench.py --rccl-one-rank --steps 20 --warmup 3 --no-cpu-baseline --no-incremental \
  --no-localize --no-fingerprint > gpurun_out/bench_rccl_one_rank_$t.json 2> gpurun_out/bench_rccl_one_rank_$t.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench_rccl_one_rank_$t.json').read().strip().splitlines()[-1]); print('rccl one rank', d['value'], d['transport'], d['split'])"
