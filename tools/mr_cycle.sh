#!/bin/bash
# GPU check of the multi-rank path: the multirank tests (all ranks on one GPU,
# host-callback transport), then the full GPU suite.  usage: bash tools/mr_cycle.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v -s --timeout 400 --timeout-method thread > gpurun_out/mr.log 2>&1 || { tail -60 gpurun_out/mr.log; exit 1; }
grep -E "PASS|FAIL|MB all-reduced" gpurun_out/mr.log | tail -20
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_multirank.py > gpurun_out/qt.log 2>&1 || { tail -40 gpurun_out/qt.log; exit 1; }
tail -2 gpurun_out/qt.log
