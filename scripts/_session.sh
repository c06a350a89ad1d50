cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v44
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
out=gpurun_out/${T}_b3chain_ab.txt
: > $out
for rep in 1 2 3; do
for cd in 0: 0:--no-b3-chain 3: 4:; do
    IFS=: read d x <<< "$cd"
    dd=""; [ $d != 0 ] && dd="--depth $d"
    f=gpurun_out/${T}_c3_d${d}${x}_$rep
    timeout -k 10 240 python -u bench.py --config c3 --steps 20 --warmup 5 $dd $x --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 scripts/depth_row.py $f.json c3 "d$d $x" | tee -a $out
done
done
