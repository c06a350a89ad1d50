# round 6: digest-pipeline (group x lanes) sweep, c2, default 4 hardware queues
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/pipe_bench.py --config c2 --sweep 16x2,24x2,32x2,12x3,16x3,20x3,32x1,48x1 --steps 96 --profile > gpurun_out/r06_v2_pipe_c2.jsonl 2> gpurun_out/r06_v2_pipe_c2.err
