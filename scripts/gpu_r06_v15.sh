# round 6 v15: same-box c2 A/B (HEAD: k_sha256<FUSED> with force-inlined helpers, vs the v9 build); c4 fused check; tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for lib in head v9; do
    if [ $lib = head ]; then L=""; else L=chunker_amd/_ab/libchunker_amd_v9.so; fi
    CHUNKER_AMD_LIB=$L timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x2 --steps 60 --profile > gpurun_out/r06_v15_c2_$lib.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/r06_v15_c2_$lib.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('c2 $lib', d['GiBps'], d['stats'].get('digest_ms_mean'))" >> gpurun_out/r06_v15_summary.txt
  done
done
B="--steps 20 --warmup 5 --no-concurrent --drop-in= --no-cpu-baseline --no-clock --no-stage-profile"
for f in 0 1; do
  timeout -k 10 300 python -u bench.py --config c4 $B --sha-fused $f > gpurun_out/r06_v15_c4_f$f.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v15_c4_f$f.json'));print('c4 fused $f', d['value'], d['pipeline']['steady_window']['GiBps'], d['roofline']['launch']['ms'])" >> gpurun_out/r06_v15_summary.txt
done
cat gpurun_out/r06_v15_summary.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -m "gpu and not slow" > gpurun_out/r06_v15_pytest.txt 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/r06_v15_pytest.txt
