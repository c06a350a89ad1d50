# round 6 v27: head-of-line probe with the real kernels' footprints: A = k_sha256-shaped
# workgroups (128 threads, 136 VGPRs, 70 KiB LDS, 30 ms), B = k_scan_flat32-shaped
# (1,024 workgroups of 512 threads, 128 VGPRs, 18 / 68 KiB LDS, 0.1 ms each)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06_v27_hol_probe.txt
P=scripts/micro/_bin/hol_probe
for g in 0 256 512 1024; do for bl in 18432 69632; do
  if [ $g = 0 ]; then timeout -k 5 30 $P 1 4 1 $bl 1 1 | tail -1 >> $O || exit $?; continue; fi
  timeout -k 5 30 $P $g 71680 30 $bl 1 1 | tail -1 >> $O || exit $?
done; done
cat $O
