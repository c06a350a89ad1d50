#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc pass per counter group; no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
TAG=${TAG:-pmc}
# STEPS: the bench's timed steps (its merged digest group is the divisor of STEPS nearest the
# default group: 20 for config 2 at STEPS=20, 2 for configs 4 / 5); no stage profile, so every
# digest launch counted is a merged one of that group
STEPS=${STEPS:-2}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$R/gpurun_out/${TAG}_$i" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps $STEPS --warmup 1 --no-cpu-baseline --no-concurrent --no-clock --no-stage-profile --e2e '' --drop-in '' > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i failed rc=$rc"; tail -5 gpurun_out/${TAG}_$i.log
    case $rc in 124|134|137|139) echo "GPU step died; stopping"; exit $rc;; esac
  fi
done
echo done
