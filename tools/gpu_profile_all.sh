# Round profiles of all three tasks (tools/gpu_profile.sh per task); summaries in gpurun_out/psum_<tag>/
set -o pipefail
cd /root/repo
TASK=FeedingJaco-v0 TAG=r03 bash tools/gpu_profile.sh > gpurun_out/prof_feeding.log 2>&1 || exit 11
TASK=ScratchItchPR2-v0 TAG=r03_scratch bash tools/gpu_profile.sh > gpurun_out/prof_scratch.log 2>&1 || exit 12
TASK=BedBathingPR2-v0 TAG=r03_bedbath bash tools/gpu_profile.sh > gpurun_out/prof_bedbath.log 2>&1 || exit 13
