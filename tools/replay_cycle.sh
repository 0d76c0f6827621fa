#!/bin/bash
# per-rank replay timings of the multi-GPU split for cfg3 at 1/2/4/8 ranks (tools/rank_replay.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/rank_replay.py replay cfg3 1 || exit 1
for n in 2 4 8; do
  timeout -k 10 300 python -u tools/rank_replay.py record cfg3 $n || exit 1
  timeout -k 10 300 python -u tools/rank_replay.py replay cfg3 $n || exit 1
done
python tools/rank_replay.py model cfg3 1 2 4 8
rm -f ${TMPDIR:-/tmp}/replay_*.npz
