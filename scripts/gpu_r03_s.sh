#!/bin/bash
# Round 3 session S: the whole GPU suite + smoke + c2 bench + kernel trace on HEAD (gpu_round.sh),
# then the c3 overlap probe: K = 1 / 2 / 4 config-3 batches in flight from K threads (does a scan
# overlapping another batch's BLAKE3 digest raise the aggregate?), and the c3 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=r03_v12 bash scripts/gpu_round.sh \
 && timeout -k 10 300 python3 bench.py --config c3 --concurrent-only --concurrent 1,2,4 > gpurun_out/r03_s_c3_conc.json 2> gpurun_out/r03_s_c3_conc.err \
 && cat gpurun_out/r03_s_c3_conc.json \
 && timeout -k 10 300 python3 bench.py --config c3 --no-concurrent > gpurun_out/r03_s_c3_bench.json 2> gpurun_out/r03_s_c3_bench.err \
 && cat gpurun_out/r03_s_c3_bench.json
rc=$?; echo "rc=$rc"; exit $rc
