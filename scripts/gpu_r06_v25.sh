# round 6 v25: head-of-line probe (scripts/micro/hol_probe.hip): does a launch with workgroups
# waiting for CU resources hold back another queue's small workgroups?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06_v25_hol_probe.txt
P=scripts/micro/_bin/hol_probe
# A: 70 KiB LDS x 128 threads (two per CU, as k_sha256), 30 ms spins; grids: fits (512), 2x, 4x
for g in 256 512 1024 2048; do for bl in 1024 18432; do
  timeout -k 5 30 $P $g 71680 30 $bl 1 | tail -1 >> $O || exit $?
done; done
# B at low priority, and A without LDS pressure (4 B) for contrast
timeout -k 5 30 $P 1024 71680 30 1024 0 | tail -1 >> $O || exit $?
timeout -k 5 30 $P 4096 4 30 1024 1 | tail -1 >> $O || exit $?
cat $O
