# round 6 v35: two boundary streams (CHUNKER_AMD_PIPE_BSTREAMS=2; with the lanes in HIP's
# low-priority pool, CHUNKER_AMD_PIPE_STREAMS=split, so every stream keeps a hardware queue):
# the lean scan takes ~1.1 ms per GiB beside the digests, so one boundary stream feeds ~20
# batches per ~23 ms -- about the rate three lanes digest.  Parity with two streams, then A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v35_summary.txt
CHUNKER_AMD_PIPE_BSTREAMS=2 CHUNKER_AMD_PIPE_STREAMS=split timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q -m "gpu and not slow" -k "pipeline" --timeout 300 --timeout-method thread > gpurun_out/r06_v35_pytest.txt 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06_v35_pytest.txt; exit 1; }
tail -1 gpurun_out/r06_v35_pytest.txt >> $S
for rep in 1 2; do
  for v in "1 high" "2 split" "1 split" "2 high"; do
    set -- $v
    CHUNKER_AMD_PIPE_BSTREAMS=$1 CHUNKER_AMD_PIPE_STREAMS=$2 timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x3,24x3,20x4 --steps 120 --profile > gpurun_out/r06_v35_$1_$2.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/r06_v35_$1_$2.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('bstreams=$1 $2', d['group'], d['lanes'], d['GiBps'], d['stats'].get('digest_ms_mean'), d.get('lat_p50_ms'))" >> $S
  done
done
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for c in c4 c5; do for v in "1 high" "2 split"; do
  set -- $v
  CHUNKER_AMD_PIPE_BSTREAMS=$1 CHUNKER_AMD_PIPE_STREAMS=$2 timeout -k 10 300 python -u bench.py --config $c $B > gpurun_out/r06_v35_${c}_$1.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v35_${c}_$1.json'));p=d['pipeline'];print('$c bstreams=$1 $2', d['value'], 'steady', p['steady_window']['GiBps'], 'launch', d['roofline']['launch']['ms'])" >> $S
done; done
cat $S
