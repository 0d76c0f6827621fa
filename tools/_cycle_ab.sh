# bit-identity digests + interleaved A/B of the default library against variant builds
mkdir -p gpurun_out
timeout -k 10 120 python tools/lib_cmp.py cfg2 cfg3 medium > gpurun_out/cmp_new.txt 2>&1 || { tail gpurun_out/cmp_new.txt; exit 1; }
cat gpurun_out/cmp_new.txt
bash tools/variant_bench.sh "$@"
