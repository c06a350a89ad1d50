#!/bin/bash
# Round 3 session AF: k_b3_fold shape sweep (groups per block / threads per block) --
# BLAKE3 tree tests on each variant, then config 3 with a kernel trace per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in prod f8_256 f32_512 f16_512 f32_256 f8_128; do
  if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
  timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "blake3_tree or group_map" > gpurun_out/r03_af_tests_$v.log 2>&1 || { echo "tests $v failed"; tail -20 gpurun_out/r03_af_tests_$v.log; exit 1; }
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_af_$v" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent > gpurun_out/r03_af_$v.json 2> gpurun_out/r03_af_$v.err || { echo "bench $v failed"; tail -3 gpurun_out/r03_af_$v.err; exit 1; }
  python3 - "$v" <<'PY'
import csv, json, sys
v = sys.argv[1]
rows = {r[0].split('(')[0].replace('void ', '').replace('cg::', ''): float(r[3]) / 1000 for r in csv.reader(open(f"gpurun_out/prof_r03_af_{v}/run_kernel_stats.csv")) if r[0] != "Name"}
line = json.loads(open(f"gpurun_out/r03_af_{v}.json").read().strip().splitlines()[-1])
print(v, line["value"], {k: round(x, 1) for k, x in rows.items() if "b3" in k})
PY
done
echo "rc=0"
