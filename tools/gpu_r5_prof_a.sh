# Round-5 profiles, part 1: FeedingJaco and ScratchItch (tools/gpu_profile.sh per task; summaries
# in gpurun_out/psum_r05*/)
set -o pipefail
cd /root/repo
TASK=FeedingJaco-v0 TAG=r05 bash tools/gpu_profile.sh > gpurun_out/prof_feeding.log 2>&1 || exit 11
TASK=ScratchItchPR2-v0 TAG=r05_scratch bash tools/gpu_profile.sh > gpurun_out/prof_scratch.log 2>&1 || exit 12
