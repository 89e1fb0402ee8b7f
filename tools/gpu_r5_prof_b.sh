# Round-5 profiles, part 2: BedBathing and DressingJaco (summaries in gpurun_out/psum_r05_*/)
set -o pipefail
cd /root/repo
TASK=BedBathingPR2-v0 TAG=r05_bedbath bash tools/gpu_profile.sh > gpurun_out/prof_bedbath.log 2>&1 || exit 13
ENVS=2048 TASK=DressingJaco-v0 TAG=r05_dressing bash tools/gpu_profile.sh > gpurun_out/prof_dressing.log 2>&1 || exit 14
