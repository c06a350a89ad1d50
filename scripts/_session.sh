cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v42
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "solo or latency_tiers or kinds_agree or digest" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
out=gpurun_out/${T}_solo_ab.txt
: > $out
for cd in c4:0,0 c4:0,200 c4:0,400 c4:0,600 c4:0,700 c5:0,0 c5:300,300 c5:400,400 c5:500,500 c2:0,0 c2:300,300; do
    IFS=: read cfg t <<< "$cd"
    f=gpurun_out/${T}_${cfg}_s${t/,/_}
    timeout -k 10 240 python -u bench.py --config $cfg --steps 20 --warmup 5 --sha-solo $t --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 scripts/depth_row.py $f.json $cfg "solo $t" | tee -a $out
done
