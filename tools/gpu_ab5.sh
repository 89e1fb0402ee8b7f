# fingerprint A/B + PR2 NcLds variants + Feeding NcLds variants
set -o pipefail
cd /root/repo && export TMPDIR=/tmp
TASKS="ScratchItchPR2-v0 BedBathingPR2-v0" VARIANTS="default nonl dnl2" bash tools/gpu_ab4.sh || exit $?
TASK=FeedingJaco-v0 VARIANTS="default fnl fnl11 fnl12" bash tools/gpu_variants.sh > gpurun_out/ab/var_FeedingJaco-v0.txt 2>&1 || exit 13
