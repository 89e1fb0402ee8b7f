# Round 5: robot Jacobians from scalar loads of the DoF links / joint types, robot parts stored as
# vectors -- fingerprints against the previous commit's build on the three tasks, interleaved
# benches of all three, and the ScratchItch phase profile.  Output: gpurun_out/r5t24/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t24
for t in 0 1 2; do
  FP_STATES=gpurun_out/r5t24/S$t.npz TASK=$t AVR_LIB=/root/repo/_ab/libavr_prev.so timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t24/old$t.npz > gpurun_out/r5t24/old$t.log 2>&1 || exit 11
  FP_STATES=gpurun_out/r5t24/S$t.npz TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t24/new$t.npz gpurun_out/r5t24/old$t.npz > gpurun_out/r5t24/new$t.log 2>&1; echo "task $t rc=$?"; tail -1 gpurun_out/r5t24/new$t.log
done
rm -f gpurun_out/r5t24/*.npz
for T in ScratchItchPR2-v0 BedBathingPR2-v0 FeedingJaco-v0; do
  TASK=$T VARIANTS="default prev" ROUNDS=2 bash tools/gpu_ab_variants.sh >> gpurun_out/r5t24/ab.log 2>&1 || exit 12
done
cat gpurun_out/r5t24/ab.log
TASK=1 timeout -k 10 300 python3 tools/prof_phases.py 512 > gpurun_out/r5t24/scratch_phases.txt 2>&1
grep -E "c_rows |nc_rows|robot_jac|minv_mul|put_robot" gpurun_out/r5t24/scratch_phases.txt | head -6
