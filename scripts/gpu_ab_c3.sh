#!/bin/bash
# A/B: config 3 (BLAKE3) bench, current build vs chunker_amd/libchunker_amd_prev.so, alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
P=$PWD/chunker_amd/libchunker_amd_prev.so
TAG=${TAG:-ab_c3}
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-concurrent > gpurun_out/${TAG}_new_$i.json 2>/dev/null || exit $?
  CHUNKER_AMD_LIB=$P timeout -k 10 200 python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-concurrent > gpurun_out/${TAG}_prev_$i.json 2>/dev/null || exit $?
done
for f in gpurun_out/${TAG}_*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['stages_ms'])"; done
