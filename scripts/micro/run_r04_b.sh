#!/bin/bash
# Round 4 session B: VALU mixes (dual issue) + SQ counters of the mixes and of the c2 pipeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 scripts/micro/_bin/issue_rates 0,3,13,100,110,111,112,113,114,115,116,117,118,119 > gpurun_out/r04_issue_mix.json 2> gpurun_out/r04_issue_mix.err || exit $?
echo "mix ok"
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d "$R/gpurun_out/r04_pmc_mix" -o run --output-format csv -- "$R/scripts/micro/_bin/issue_rates" 0,3,100,110,114,115 > gpurun_out/r04_pmc_mix.log 2>&1 || exit $?
echo "pmc mix ok"
timeout -k 10 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS -d "$R/gpurun_out/r04pmcsq_1" -o run --output-format csv -- python3 "$R/bench.py" --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r04pmcsq_1.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_WAVES -d "$R/gpurun_out/r04pmcsq_2" -o run --output-format csv -- python3 "$R/bench.py" --config c2 --steps 2 --warmup 1 --no-cpu-baseline --no-concurrent --e2e '' > gpurun_out/r04pmcsq_2.log 2>&1 || exit $?
python3 scripts/pmc_summary.py gpurun_out r04pmcsq > gpurun_out/r04_pmc_sq_c2.json
echo "rc=0"
