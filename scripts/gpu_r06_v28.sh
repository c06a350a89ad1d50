# round 6 v28: which scan shape fits beside two k_sha256-shaped workgroups per CU:
# 512 threads x 128 VGPRs (real 1), 256 threads x 128 VGPRs (real 2), 512 x 112 (real 3);
# scan LDS 18 KiB (lean table) or 68 KiB
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=gpurun_out/r06_v28_hol_probe.txt
P=scripts/micro/_bin/hol_probe
for real in 1 2 3; do for bl in 17408 69632; do
  timeout -k 5 30 $P 512 71680 30 $bl 1 $real | tail -1 >> $O || exit $?
done; done
cat $O
