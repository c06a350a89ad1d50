#!/bin/bash
# Round 3 session AG: packed BLAKE3 leaves (k_b3_leaves: the leaves of all chunks back to
# back, 64 per wave) -- BLAKE3 parity tests + fuzz, then config 3 alternating the product
# (packed) with the one-group-per-wave build (CG_B3_PACKED=0), kernel traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py -k "blake3 or B3 or b3 or config3 or group_map or fuzz" > gpurun_out/r03_ag_tests.log 2>&1 || { tail -30 gpurun_out/r03_ag_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_ag_tests.log)"
for r in 1 2; do
  for v in prod unpacked; do
    if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_ag_${v}_$r" -o run --output-format csv -- python3 "$R/bench.py" --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent > gpurun_out/r03_ag_${v}_$r.json 2> gpurun_out/r03_ag_${v}_$r.err || { tail -3 gpurun_out/r03_ag_${v}_$r.err; exit 1; }
    timeout -k 10 200 python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-concurrent > gpurun_out/r03_ag_${v}_$r.bench.json 2> gpurun_out/r03_ag_${v}_$r.bench.err || exit 1
    python3 - "$v" "$r" <<'PY'
import csv, json, sys
v, r = sys.argv[1], sys.argv[2]
rows = {x[0].split('(')[0].replace('void ', '').replace('cg::', ''): float(x[3]) / 1000 for x in csv.reader(open(f"gpurun_out/prof_r03_ag_{v}_{r}/run_kernel_stats.csv")) if x[0] != "Name"}
line = json.loads(open(f"gpurun_out/r03_ag_{v}_{r}.bench.json").read().strip().splitlines()[-1])
print(v, r, line["value"], line["stages_ms"]["digest_timed"], {k: round(x, 1) for k, x in rows.items() if "b3" in k})
PY
  done
done
echo "rc=0"
