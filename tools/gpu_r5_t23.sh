# Round 5: the second robot endpoint of a contact row added in registers (no read-back of the
# first from memory) -- fingerprints against the previous commit's build (_ab/libavr_prev.so) on
# shared initial states for the three tasks, and interleaved PR2 benches.  Output: gpurun_out/r5t23/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t23
for t in 0 1 2; do
  FP_STATES=gpurun_out/r5t23/S$t.npz TASK=$t AVR_LIB=/root/repo/_ab/libavr_prev.so timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t23/old$t.npz > gpurun_out/r5t23/old$t.log 2>&1 || exit 11
  FP_STATES=gpurun_out/r5t23/S$t.npz TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t23/new$t.npz gpurun_out/r5t23/old$t.npz > gpurun_out/r5t23/new$t.log 2>&1; echo "task $t rc=$?"; tail -1 gpurun_out/r5t23/new$t.log
done
rm -f gpurun_out/r5t23/*.npz
for T in ScratchItchPR2-v0 BedBathingPR2-v0; do
  TASK=$T VARIANTS="default prev" ROUNDS=2 bash tools/gpu_ab_variants.sh >> gpurun_out/r5t23/ab.log 2>&1 || exit 12
done
cat gpurun_out/r5t23/ab.log
