set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/ab
for T in FeedingJaco-v0 ScratchItchPR2-v0; do
  TASK=$T VARIANTS="default nofp" bash tools/gpu_variants.sh > gpurun_out/ab/var_fp_$T.txt 2>&1 || exit 11
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ab/pytest_fp.log 2>&1 || exit 12
