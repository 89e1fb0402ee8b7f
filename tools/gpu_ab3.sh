# Variant benches for all three tasks (exp/libavr_<v>.so), then the GPU suite on the shipped build.
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/var
for T in ScratchItchPR2-v0 BedBathingPR2-v0 FeedingJaco-v0; do
  TASK=$T VARIANTS="${VARIANTS:-default}" bash tools/gpu_variants.sh > gpurun_out/var/$T.txt 2>&1 || exit 11
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/var/pytest.log 2>&1 || exit 12
