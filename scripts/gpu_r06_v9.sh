# round 6 v9: PMC of k_sha256 on config 4 for the product (4-slot ring, 2 workgroups per CU)
# and the 2-slot ring at 4 per CU; kernel trace + PMC traffic of the config-2 pipeline bench
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
G2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"
G3="FETCH_SIZE"
G4="WRITE_SIZE"
pass() {  # tag lib occ cfg counters...
  local tag=$1 lib=$2 occ=$3 cfg=$4; shift 4
  CHUNKER_AMD_LIB=$lib timeout -k 10 240 rocprofv3 --pmc "$@" -d "$R/gpurun_out/$tag" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 4 --warmup 1 --group 1 --lanes 1 --no-cpu-baseline --no-concurrent --no-clock --e2e= --drop-in= --no-stage-profile --sha-occ $occ > gpurun_out/$tag.log 2>&1
}
i=0
for v in "prod::2,2" "ring2:$R/chunker_amd/_ab/libchunker_amd_ring2.so:4,4"; do
  name=${v%%:*}; rest=${v#*:}; lib=${rest%%:*}; occ=${rest#*:}
  for g in "$G1" "$G2" "$G3" "$G4"; do
    i=$((i+1))
    pass r06_v9_pmc_c4_${name}_$i "$lib" $occ c4 $g || { rc=$?; echo "pass $i rc=$rc"; tail -3 gpurun_out/r06_v9_pmc_c4_${name}_$i.log; case $rc in 124|134|137|139) exit $rc;; esac; }
  done
done
# config 2 product bench under the kernel trace (the timed command minus the extra legs)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06_v9_trace_c2" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-concurrent --e2e= --drop-in= --no-clock --no-stage-profile > gpurun_out/r06_v9_trace_c2.json 2> gpurun_out/r06_v9_trace_c2.err || echo "trace rc=$?"
for g in "$G3" "$G4"; do
  i=$((i+1))
  CHUNKER_AMD_LIB= timeout -k 10 240 rocprofv3 --pmc $g -d "$R/gpurun_out/r06_v9_pmc_c2_$i" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-concurrent --e2e= --drop-in= --no-clock --no-stage-profile > gpurun_out/r06_v9_pmc_c2_$i.log 2>&1 || echo "c2 pmc rc=$?"
done
echo done
