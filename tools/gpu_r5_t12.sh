# Round 5: the whole GPU suite on the GJK change (stalled lane GJK pairs rerun in double), then
# interleaved benches of the three tasks against the previous build (_ab/libavr_head.so).
# Output: gpurun_out/r5t12/, gpurun_out/ab/
set -o pipefail
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r5t12
timeout -k 10 900 python3 -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests/ > gpurun_out/r5t12/pytest_gpu.log 2>&1
rc=$?; echo tests rc=$rc; case $rc in 124|134|137|139) exit $rc ;; esac
VARIANTS="default head" ROUNDS=2 bash tools/gpu_ab_variants.sh > gpurun_out/r5t12/ab.log 2>&1 || exit 22
for T in ScratchItchPR2-v0 BedBathingPR2-v0; do
  TASK=$T VARIANTS="default head" ROUNDS=2 bash tools/gpu_ab_variants.sh >> gpurun_out/r5t12/ab.log 2>&1 || exit 23
done
