# round 6 v29: the scans of the digest pipeline's boundary stream wait ~0.5-26 ms for CU room
# under the merged SHA-256 launches: a 512-thread, 128-VGPR scan workgroup cannot be placed
# on a CU holding two k_sha256 workgroups (per-SIMD register packing, profiles/r06_v28_*), a
# 256-thread one with an 18 KiB table can.  A/B: CHUNKER_AMD_SCAN_LEAN=1 (one-shot flat scan
# with 8 table copies, 256 threads) vs the product, same box; parity first.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
S=gpurun_out/r06_v29_summary.txt
CHUNKER_AMD_SCAN_LEAN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q -m "gpu and not slow" --timeout 300 --timeout-method thread > gpurun_out/r06_v29_pytest_lean.txt 2>&1 || { echo "lean tests failed"; tail -30 gpurun_out/r06_v29_pytest_lean.txt; exit 1; }
tail -1 gpurun_out/r06_v29_pytest_lean.txt >> $S
for rep in 1 2; do
  for lean in 0 1; do
    CHUNKER_AMD_SCAN_LEAN=$lean timeout -k 10 300 python -u scripts/pipe_bench.py --config c2 --sweep 20x2,20x3,24x2 --steps 60 --profile > gpurun_out/r06_v29_c2_l$lean.jsonl 2>/dev/null || exit $?
    python3 -c "
import json
for l in open('gpurun_out/r06_v29_c2_l$lean.jsonl'):
    d=json.loads(l)
    if 'group' in d: print('c2 lean=$lean', d['group'], d['lanes'], d['GiBps'], d['stats'].get('digest_ms_mean'), d.get('lat_p50_ms'))" >> $S
  done
done
B="--steps 20 --warmup 5 --no-concurrent --e2e= --drop-in= --no-cpu-baseline --no-clock"
for lean in 0 1; do
  CHUNKER_AMD_SCAN_LEAN=$lean timeout -k 10 300 python -u bench.py $B > gpurun_out/r06_v29_c2_bench_l$lean.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/r06_v29_c2_bench_l$lean.json'));print('c2 bench lean=$lean', d['value'], 'scan_ms', d['stages_ms']['scan'], 'cold', d['roofline']['scan_kernel']['cold_hbm']['ms'], 'launch', d['roofline']['launch']['ms'])" >> $S
done
cat $S
CHUNKER_AMD_SCAN_LEAN=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/r06_v29_trace" -o run --output-format csv -- python3 "$R/scripts/pipe_bench.py" --config c2 --sweep 20x3 --steps 60 --profile > gpurun_out/r06_v29_trace.jsonl 2> gpurun_out/r06_v29_trace.err || exit $?
python3 - <<'PY'
import csv, glob, collections
import numpy as np
f = glob.glob('gpurun_out/r06_v29_trace/*kernel_trace.csv')[0]
byk = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    byk[r['Kernel_Name'].split('(')[0].replace('void ', '')].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for n, v in sorted(byk.items(), key=lambda x: -sum(x[1]))[:4]:
    v = np.array(v); print('lean256 trace', n[:50], len(v), 'mean %.3f p50 %.3f max %.3f' % (v.mean(), np.median(v), v.max()))
PY
