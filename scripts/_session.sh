cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v45
for rep in 1 2; do
for pr in 0 1; do
f=gpurun_out/${T}_e2e_prio${pr}_$rep
CG_BENCH_COPY_PRIO=$pr timeout -k 10 400 python -u bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline --concurrent 1 --e2e 1 --drop-in '' --no-clock > $f.json 2> $f.err || exit $?
python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));e=d['concurrent']['e2e'];print('prio', sys.argv[2], d['value'], e['h2d_only'], e['K1'], e['one_caller_overlapped']['GiBps'])" $f.json $pr
done
done
