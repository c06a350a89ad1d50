# round 6 v13: same-box c2 A/B (HEAD vs the pre-fused v9 build) through scripts/pipe_bench.py, then the whole GPU suite
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for lib in head v9; do
    if [ $lib = head ]; then L=""; else L=chunker_amd/_ab/libchunker_amd_v9.so; fi
    CHUNKER_AMD_LIB=$L timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x2 --steps 60 --profile > gpurun_out/r06_v13_c2_$lib.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/r06_v13_c2_$lib.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('$lib', d['GiBps'], d['stats'].get('digest_ms_mean'))" >> gpurun_out/r06_v13_summary.txt
  done
done
cat gpurun_out/r06_v13_summary.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_v13_gpu_suite.txt 2>&1
echo "suite rc=$?"; tail -5 gpurun_out/r06_v13_gpu_suite.txt
