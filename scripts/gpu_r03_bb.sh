#!/bin/bash
# Round 3 session BB: SHA-256 LDS ring depth 2 / 3 vs 4 (product) with the round code aligned:
# config 4 (GPU-filling, one-lane tier throughput) and config 2, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for cfg in c4 c2; do
    for v in prod ring2 ring3; do
      if [ $v = prod ]; then unset CHUNKER_AMD_LIB; else export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so; fi
      timeout -k 10 300 python3 bench.py --config $cfg --steps 8 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_bb_${cfg}_${v}_$r.json 2> gpurun_out/r03_bb_${cfg}_${v}_$r.err || { tail -3 gpurun_out/r03_bb_${cfg}_${v}_$r.err; exit 1; }
      python3 -c "
import json; l=json.loads(open('gpurun_out/r03_bb_${cfg}_${v}_$r.json').read().strip().splitlines()[-1])
print('$cfg', '$v', $r, l['value'], l['stages_ms']['digest_timed'])" | tee -a gpurun_out/r03_bb_ab.txt
    done
  done
done
echo "rc=0"
