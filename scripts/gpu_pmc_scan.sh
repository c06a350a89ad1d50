#!/bin/bash
# PMC passes over the scan diagnostic (one mode, config c2); one rocprofv3 pass per counter group.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
MODE=${MODE:-3}
TAG=${TAG:-pmcscan}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM" \
           "GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d "$R/gpurun_out/${TAG}_$i" -o run --output-format csv -- python3 "$R/scripts/diag_scan.py" --modes $MODE --configs c2 --no-pattern > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc"; tail -5 gpurun_out/${TAG}_$i.log; exit $rc; fi
done
echo done
