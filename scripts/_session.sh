cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r05_v43
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "async or pipeline" > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
out=gpurun_out/${T}_detached_ab.txt
: > $out
for rep in 1 2; do
for cd in 4:0: 4:0:--join-stream 4:4: 4:4:--join-stream 16:0: 16:0:--join-stream; do
    IFS=: read q d j <<< "$cd"
    dd=""; [ $d != 0 ] && dd="--depth $d"
    f=gpurun_out/${T}_q${q}_d${d}${j}_$rep
    timeout -k 10 240 python -u bench.py --config c2 --steps 20 --warmup 5 --hw-queues $q $dd $j --no-cpu-baseline \
      --no-concurrent --drop-in '' --e2e '' --no-clock > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 scripts/depth_row.py $f.json c2 "q$q d$d $j" | tee -a $out
done
done
