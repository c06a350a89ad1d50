#!/bin/bash
# Round 3 session BL: the two-block consumer body for the one-lane tier too (c4's throughput
# tier) vs the product -- SHA parity tests on the variant, configs 4 / 2 alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_lanebody.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py > gpurun_out/r03_bl_tests.log 2>&1 || { tail -30 gpurun_out/r03_bl_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_bl_tests.log)"
for r in 1 2 3; do
  for cfg in c4 c2; do
    for v in prod lanebody; do
      if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
      timeout -k 10 300 python3 bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_bl_${cfg}_${v}_$r.json 2> gpurun_out/r03_bl_${cfg}_${v}_$r.err || { tail -3 gpurun_out/r03_bl_${cfg}_${v}_$r.err; exit 1; }
      python3 -c "
import json; l=json.loads(open('gpurun_out/r03_bl_${cfg}_${v}_$r.json').read().strip().splitlines()[-1])
print('$cfg', '$v', $r, l['value'], l['stages_ms']['digest_timed'])" | tee -a gpurun_out/r03_bl_ab.txt
    done
  done
done
echo "rc=0"
