#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc pass per counter group; no trace domains).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-c3}
TAG=${TAG:-pmc}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp -d "$R/gpurun_out/${TAG}_$i" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --steps 2 --warmup 1 --no-cpu-baseline --no-concurrent --no-clock --e2e '' --drop-in '' > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then
    echo "pass $i failed rc=$rc"; tail -5 gpurun_out/${TAG}_$i.log
    case $rc in 124|134|137|139) echo "GPU step died; stopping"; exit $rc;; esac
  fi
done
echo done
