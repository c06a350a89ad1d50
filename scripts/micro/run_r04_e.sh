#!/bin/bash
# Round 4 session E: persistent scan without the exit L2 flush, coalescer set counts,
# and the single-GPU --dist-force overhead check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r04e_pytest_fast.log 2>&1 || { tail -40 gpurun_out/r04e_pytest_fast.log; exit 1; }
tail -2 gpurun_out/r04e_pytest_fast.log
timeout -k 10 300 python -u scripts/scan_ab.py --configs c2,c4,c5 --reps 5 --grids 0,256,512 > gpurun_out/r04e_scan_ab.json 2> gpurun_out/r04e_scan_ab.err || { tail -5 gpurun_out/r04e_scan_ab.err; exit 1; }
for v in spu4 spu16; do
  CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so timeout -k 10 300 python -u scripts/scan_ab.py --configs c2,c4,c5 --reps 5 --kernels 0 > gpurun_out/r04e_scan_ab_$v.json 2> gpurun_out/r04e_scan_ab_$v.err || { tail -5 gpurun_out/r04e_scan_ab_$v.err; exit 1; }
done
for k in 1 2 3; do
  CHUNKER_AMD_COAL_SETS=$k timeout -k 10 300 python bench.py --concurrent-only --concurrent-reps 6 > gpurun_out/r04e_conc_coal$k.json 2> gpurun_out/r04e_conc_coal$k.err || exit 1
done
timeout -k 10 300 python bench.py --concurrent-only --concurrent-reps 6 --no-coalesce > gpurun_out/r04e_conc_nocoal.json 2> gpurun_out/r04e_conc_nocoal.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-concurrent --e2e '' --no-clock > gpurun_out/r04e_bench_c2.json 2> gpurun_out/r04e_bench_c2.err || exit 1
cat gpurun_out/r04e_conc_coal1.json gpurun_out/r04e_conc_coal2.json gpurun_out/r04e_conc_coal3.json gpurun_out/r04e_conc_nocoal.json gpurun_out/r04e_scan_ab.json gpurun_out/r04e_scan_ab_spu4.json gpurun_out/r04e_scan_ab_spu16.json | cut -c1-1800
cut -c1-400 gpurun_out/r04e_bench_c2.json
echo "rc=0"
