# round 6 v4: queue probe with busy fillers, BLAKE3 pipeline debug
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/micro/queue_probe.sh > gpurun_out/r06_v4_queue_probe.txt 2>&1
timeout -k 10 200 python -u scripts/debug_b3_pipe.py > gpurun_out/r06_v4_debug_b3.txt 2>&1
echo rc=$?
