# Round profiles of every task (tools/gpu_profile.sh per task); summaries in gpurun_out/psum_<tag>/
set -o pipefail
cd /root/repo
R=${ROUND:-r04}
TASK=FeedingJaco-v0 TAG=$R bash tools/gpu_profile.sh > gpurun_out/prof_feeding.log 2>&1 || exit 11
TASK=ScratchItchPR2-v0 TAG=${R}_scratch bash tools/gpu_profile.sh > gpurun_out/prof_scratch.log 2>&1 || exit 12
TASK=BedBathingPR2-v0 TAG=${R}_bedbath bash tools/gpu_profile.sh > gpurun_out/prof_bedbath.log 2>&1 || exit 13
ENVS=2048 TASK=DressingJaco-v0 TAG=${R}_dressing bash tools/gpu_profile.sh > gpurun_out/prof_dressing.log 2>&1 || exit 14
