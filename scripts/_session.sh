cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v32
for rep in 1 2; do
for cd in 1:0 10:0 10:1 10:3; do
    IFS=: read d r <<< "$cd"
    f=gpurun_out/${T}_c2_d${d}_rest${r}_$rep
    timeout -k 10 240 python -u bench.py --config c2 --steps 20 --warmup 5 --depth $d --profile-rest $r --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || exit $?
    python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], d['value'], d['stages_ms']['scan'], d['roofline']['scan_kernel']['cold_hbm']['ms'])" $f.json
done
done
