#!/bin/bash
# Round 3 session AI: batched branch-free warm-up verification in k_walk (CG_VERIFY_U
# chunks per lane per pass) -- the GPU parity suite + fuzz, then configs 4/5/3 walk stage
# for the product (U=4) against the previous build (old) and U=2 / U=8.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py > gpurun_out/r03_ai_tests.log 2>&1 || { tail -30 gpurun_out/r03_ai_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/r03_ai_tests.log)"
for cfg in c4 c5 c3; do
  for r in 1 2; do
    for v in prod old u2 u8; do
      if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
      timeout -k 10 200 python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_ai_${cfg}_${v}_$r.json 2> gpurun_out/r03_ai_${cfg}_${v}_$r.err || { tail -3 gpurun_out/r03_ai_${cfg}_${v}_$r.err; exit 1; }
      python3 -c "
import json; l=json.loads(open('gpurun_out/r03_ai_${cfg}_${v}_$r.json').read().strip().splitlines()[-1])
print('$cfg', '$v', $r, l['value'], l['ms_per_step'], l['stages_ms'])" | tee -a gpurun_out/r03_ai_ab.txt
    done
  done
done
echo "rc=0"
