#!/bin/bash
# Round 3 session AP: kernel traces of configs 4 and 5 on HEAD (walk-stage split between
# k_walk_pieces and k_walk after the v30 verification change).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r03_v35_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/prof_r03_v35_$cfg.log 2>&1 || exit 1
  echo "$cfg ok"
done
echo "rc=0"
