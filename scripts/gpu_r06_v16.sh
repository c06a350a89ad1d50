# round 6 v16: fused tier removed (k_sha256 back to the v9 code, instruction for instruction):
# same-box c2 A/B against the v9 build, c4 / c5 lines, parity + pipeline tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
S=gpurun_out/r06_v16_summary.txt
for rep in 1 2; do
  for lib in head v9; do
    if [ $lib = head ]; then L=""; else L=chunker_amd/_ab/libchunker_amd_v9.so; fi
    CHUNKER_AMD_LIB=$L timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x2 --steps 60 --profile > gpurun_out/r06_v16_c2_$lib.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/r06_v16_c2_$lib.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('c2 $lib', d['GiBps'], d['stats'].get('digest_ms_mean'))" >> $S
  done
done
B="--steps 20 --warmup 5 --no-concurrent --drop-in= --no-cpu-baseline --no-clock --no-stage-profile"
for c in c4 c5; do
  timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v16_$c.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v16_$c.json'));print('$c', d['value'], d['pipeline']['steady_window']['GiBps'], d['roofline']['launch']['ms'], d['pipeline']['sha_wgs_per_cu'])" >> $S
done
cat $S
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -m "gpu and not slow" > gpurun_out/r06_v16_pytest.txt 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r06_v16_pytest.txt
