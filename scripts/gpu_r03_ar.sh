#!/bin/bash
# Round 3 session AR: scan run length (segments per wave, cap 32 in the product) on the
# 16 GiB configs 4 / 5 and the 1 GiB config 3, alternating builds on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for cfg in c4 c3; do
    for v in base spw64 spw128; do
      export CHUNKER_AMD_LIB=chunker_amd/_ab/libchunker_amd_$v.so
      timeout -k 10 300 python3 bench.py --config $cfg --steps 6 --warmup 2 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r03_as_${cfg}_${v}_$r.json 2> gpurun_out/r03_as_${cfg}_${v}_$r.err || { tail -3 gpurun_out/r03_as_${cfg}_${v}_$r.err; exit 1; }
      python3 -c "
import json; l=json.loads(open('gpurun_out/r03_as_${cfg}_${v}_$r.json').read().strip().splitlines()[-1])
print('$cfg', '$v', $r, l['value'], l['stages_ms']['scan'], l['roofline'].get('scan_kernel',{}).get('frac'))" | tee -a gpurun_out/r03_as_ab.txt
    done
  done
done
echo "rc=0"
