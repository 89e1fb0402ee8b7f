# Bit-identity of the working tree's kernels against the previous build (_old/, built beforehand),
# all three tasks on shared initial states; then variant benches (VARIANTS) for TASKS.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
for t in 0 1 2; do
  FP_STATES=gpurun_out/ab/S$t.npz TASK=$t AVR_FP_ROOT=/root/repo/_old timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/ab/old$t.npz > gpurun_out/ab/old$t.log 2>&1 || exit 11
  FP_STATES=gpurun_out/ab/S$t.npz TASK=$t timeout -k 10 240 python3 tools/fingerprint.py gpurun_out/ab/new$t.npz gpurun_out/ab/old$t.npz > gpurun_out/ab/new$t.log 2>&1; echo "task $t rc=$?"; tail -1 gpurun_out/ab/new$t.log
done
rm -f gpurun_out/ab/*.npz
for T in ${TASKS:-ScratchItchPR2-v0}; do
  [ "$T" = none ] && continue
  TASK=$T VARIANTS="${VARIANTS:-default}" bash tools/gpu_variants.sh > gpurun_out/ab/var_$T.txt 2>&1 || exit 12
done
