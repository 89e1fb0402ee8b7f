# Round 5: kernel a stages the joint tables (joint types, subtree masks, DoF links) in LDS --
# fingerprints against the previous commit's build on three tasks (tools/fingerprint.py has no
# DressingJaco scene: its GPU parity tests instead), interleaved benches.
# Output: gpurun_out/r5t25/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t25
for t in ${FP_TASKS-0 1 2}; do
  FP_STATES=gpurun_out/r5t25/S$t.npz TASK=$t AVR_LIB=/root/repo/_ab/libavr_prev.so timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t25/old$t.npz > gpurun_out/r5t25/old$t.log 2>&1 || exit 11
  FP_STATES=gpurun_out/r5t25/S$t.npz TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/r5t25/new$t.npz gpurun_out/r5t25/old$t.npz > gpurun_out/r5t25/new$t.log 2>&1; echo "task $t rc=$?"; tail -1 gpurun_out/r5t25/new$t.log
done
rm -f gpurun_out/r5t25/*.npz
for T in FeedingJaco-v0 ScratchItchPR2-v0 BedBathingPR2-v0 DressingJaco-v0; do
  TASK=$T VARIANTS="default prev" ROUNDS=2 bash tools/gpu_ab_variants.sh >> gpurun_out/r5t25/ab.log 2>&1 || exit 12
done
cat gpurun_out/r5t25/ab.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -k 'ressing' -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5t25/dressing_tests.log 2>&1; echo "dressing tests rc=$?"; tail -2 gpurun_out/r5t25/dressing_tests.log
