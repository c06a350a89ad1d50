# round 6: queue probe + first digest-pipeline sweep (c2, default 4 hardware queues)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/micro/queue_probe.sh > gpurun_out/r06_v1_queue_probe.txt 2>&1 || true
timeout -k 10 500 python -u scripts/pipe_bench.py --config c2 --sweep 4x2,8x2,16x1,16x2 --steps 48 --check > gpurun_out/r06_v1_pipe_c2.jsonl 2> gpurun_out/r06_v1_pipe_c2.err
